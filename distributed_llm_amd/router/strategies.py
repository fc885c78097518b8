"""The five routing strategies (token / semantic / heuristic / hybrid / perf).

Behavioural spec: SURVEY §2.9; reference ``src/query_router_engine.py``:
  token     :82-107   semantic :114-213   heuristic :220-364
  hybrid    :371-414  perf     :421-458
Decisions, confidences, method strings and reasoning formats are reproduced exactly so
routing accuracy and CSV columns are comparable with the reference.

Differences by design (not behaviour):
  * embedders are shared singletons (``embedder.get_embedder``) instead of one
    SentenceTransformer per router instance;
  * centroid similarity goes through ``CentroidScorer`` which runs the fused HIP cosine
    kernel when the query embedding lives on the GPU;
  * ``PerformanceAwareRouter`` keeps running sums (O(1) score) and is lock-protected.
"""
from __future__ import annotations

import json
import os
import re
import threading
from collections import deque
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..config import LARGE, SMALL
from . import tokens as _tokens
from .embedder import Embedder, get_embedder


@dataclass
class RoutingDecision:
    """Reference ``RoutingDecision`` (``query_router_engine.py:55-62``)."""
    device: str
    confidence: float
    method: str
    reasoning: str
    complexity_score: Optional[float] = None
    cache_hit: bool = False


class BaseRouter:
    name = "base"

    def __init__(self, config: Dict[str, Any]):
        self.config = config

    def route(self, query: str, context: Optional[str] = None) -> RoutingDecision:
        raise NotImplementedError


# ----------------------------------------------------------------------------- token

class TokenBasedRouter(BaseRouter):
    name = "token"

    def __init__(self, config: Dict[str, Any]):
        super().__init__(config)
        self.threshold = int(config.get("token_threshold", 1000))
        self.model = config.get("model", "meta-llama/Llama-2-7b-hf")

    def count(self, query: str, context: Optional[str]) -> int:
        text = f"{context}\n{query}" if context else query
        return int(_tokens.count_text(text))

    def route(self, query: str, context: Optional[str] = None) -> RoutingDecision:
        n = self.count(query, context)
        thr = self.threshold
        return RoutingDecision(
            device=LARGE if n > thr else SMALL,
            confidence=float(min(abs(n - thr) / max(thr, 1), 1.0)),
            method="token",
            reasoning=f"tokens={n} threshold={thr}",
            complexity_score=float(n),
        )


# ----------------------------------------------------------------------------- semantic

_SEED_TEXTS = {
    SMALL: ["Hello", "What is 2+2?", "Define machine learning", "What is the weather today?"],
    LARGE: [
        "Write a Python function to solve knapsack and explain time complexity",
        "Analyze the economic impact of climate policy with trade-offs",
        "Draft a detailed report with methodology and evaluation plan",
        "Explain quantum computing implications for cryptography in depth",
    ],
}


def load_label_texts(path: str) -> Tuple[List[str], List[str]]:
    """Read centroid training texts.

    Accepts the reference format (list of ``{"text", "label"}``, labels nano/orin) and this
    repo's grouped format (``{"small": [...], "large": [...]}``).
    """
    with open(path, "r", encoding="utf-8") as f:
        data = json.load(f)
    small: List[str] = []
    large: List[str] = []
    if isinstance(data, dict):
        for key, bucket in (("small", small), ("nano", small), ("large", large), ("orin", large)):
            for t in data.get(key, []) or []:
                t = (t or "").strip()
                if t:
                    bucket.append(t)
    else:
        for row in data:
            text = (row.get("text") or "").strip()
            label = (row.get("label") or "").strip().lower()
            if not text:
                continue
            if label in ("nano", "small"):
                small.append(text)
            elif label in ("orin", "large"):
                large.append(text)
    return small, large


class CentroidScorer:
    """Cosine similarity of query embeddings against a small centroid table.

    Host path: numpy.  Device path: ``ops.cosine_scores`` (fused normalise + GEMV HIP kernel).
    """

    def __init__(self, centroids: np.ndarray):
        self.centroids = np.asarray(centroids, dtype=np.float32)
        self._dev = None

    def scores(self, q: Any) -> np.ndarray:
        if not isinstance(q, np.ndarray):  # device tensor
            from .. import ops
            if self._dev is None or self._dev.device != q.device:
                import torch
                self._dev = torch.from_numpy(self.centroids).to(q.device)
            return ops.cosine_scores(q.reshape(1, -1).float(), self._dev).reshape(-1).cpu().numpy()
        out = np.zeros(len(self.centroids), dtype=np.float64)
        nq = float(np.linalg.norm(q))
        for i, c in enumerate(self.centroids):
            nc = float(np.linalg.norm(c))
            out[i] = 0.0 if (nq < 1e-9 or nc < 1e-9) else float(np.dot(q, c) / (nq * nc))
        return out

    def scores_batch(self, qs: Any) -> np.ndarray:
        """[n, n_centroids] for a batch of embeddings: ONE kernel launch and one copy back on the
        device path (row i equals ``scores(qs[i])``: the kernel scores rows independently)."""
        if isinstance(qs, np.ndarray):
            return np.stack([self.scores(q) for q in qs]) if len(qs) else np.zeros((0, len(self.centroids)))
        from .. import ops
        if self._dev is None or self._dev.device != qs.device:
            import torch
            self._dev = torch.from_numpy(self.centroids).to(qs.device)
        return ops.cosine_scores(qs.reshape(qs.shape[0], -1).float(), self._dev).cpu().numpy()


class SemanticRouter(BaseRouter):
    name = "semantic"

    def __init__(self, config: Dict[str, Any], embedder: Optional[Embedder] = None):
        super().__init__(config)
        self.embedder = embedder or get_embedder(config.get("embedding_model", "all-MiniLM-L6-v2"))
        self.label_path = config.get("semantic_label_path", "")
        self.margin_threshold = float(config.get("semantic_margin_threshold", 0.03))
        self.min_similarity = float(config.get("semantic_min_similarity", 0.05))
        self._token_fallback = TokenBasedRouter(config)
        self.nano_center, self.orin_center = self._build_centroids(self.label_path)
        self._scorer = CentroidScorer(np.stack([self.nano_center, self.orin_center]))
        self._score_memo: Dict[str, Tuple[float, float]] = {}   # this routing batch's scores (prefetch)

    def _build_centroids(self, label_path: str) -> Tuple[np.ndarray, np.ndarray]:
        if not label_path or not os.path.exists(label_path):
            small, large = _SEED_TEXTS[SMALL], _SEED_TEXTS[LARGE]
        else:
            small, large = load_label_texts(label_path)
            if len(small) < 3 or len(large) < 3:
                raise ValueError(
                    f"Need >=3 samples per class. Got nano={len(small)} orin={len(large)}")
        return (np.mean(self.embedder.encode(small), axis=0),
                np.mean(self.embedder.encode(large), axis=0))

    def prefetch(self, queries: List[str]) -> None:
        """Score a whole routing batch against the centroids in one launch (the orchestrator calls
        this after the batched encoder prefetch); ``similarities`` then reads the batch's scores
        instead of launching a kernel and syncing per query.  Same values: the embeddings come
        from the same encoder memo / batch scope, and the kernel scores rows independently."""
        enc_t = getattr(self.embedder, "encode_tensor", None)
        if enc_t is None or not queries:
            return
        qs = list(dict.fromkeys(queries))
        sc = self._scorer.scores_batch(enc_t(qs))
        self._score_memo = {q: (float(a), float(b)) for q, (a, b) in zip(qs, sc)}

    def similarities(self, query: str, q_emb: Any = None) -> Tuple[float, float]:
        if q_emb is None:
            hit = self._score_memo.get(query)
            if hit is not None:
                return hit
            enc_t = getattr(self.embedder, "encode_tensor", None)
            q_emb = enc_t([query])[0] if enc_t is not None else self.embedder.encode([query])[0]
        s = self._scorer.scores(q_emb)
        return float(s[0]), float(s[1])

    def route(self, query: str, context: Optional[str] = None, q_emb: Any = None) -> RoutingDecision:
        sim_n, sim_o = self.similarities(query, q_emb)
        if sim_n < self.min_similarity and sim_o < self.min_similarity:
            d = self._token_fallback.route(query, context)
            return RoutingDecision(
                device=d.device, confidence=d.confidence * 0.5,
                method="semantic_fallback_irrelevant",
                reasoning=f"low similarity (n={sim_n:.2f}, o={sim_o:.2f}) -> {d.reasoning}",
                complexity_score=float(sim_o))
        margin = abs(sim_o - sim_n)
        if margin < self.margin_threshold:
            d = self._token_fallback.route(query, context)
            return RoutingDecision(
                device=d.device, confidence=float(margin),
                method="semantic_fallback_ambiguous",
                reasoning=(f"ambiguous margin={margin:.3f} (n={sim_n:.2f}, o={sim_o:.2f}) "
                           f"-> {d.reasoning}"),
                complexity_score=float(sim_o))
        return RoutingDecision(
            device=LARGE if sim_o > sim_n else SMALL,
            confidence=float(min(1.0, margin / 0.2)),
            method="semantic",
            reasoning=f"sim_nano={sim_n:.3f} sim_orin={sim_o:.3f} margin={margin:.3f}",
            complexity_score=float(sim_o))


# ----------------------------------------------------------------------------- heuristic

# (category, [regex...]) in evaluation order; matched against the lower-cased query.
COMPLEX_RULES: List[Tuple[str, List[str]]] = [
    ("code_build_debug", [
        r"\b(write|implement|code|program|script|build|refactor|debug|fix)\b",
        r"\b(traceback|exception|error|segfault|timeout|hanging)\b",
        r"\b(api|flask|fastapi|docker|kubernetes|ssh|tunnel|nginx)\b",
        r"\b(system design|architecture|distributed|scalability|load balanc)\b"]),
    ("math_cs_theory", [
        r"\b(prove|lemma|theorem|corollary|derivative|integral|gradient)\b",
        r"\b(time complexity|space complexity|big[- ]o)\b",
        r"\b(dynamic programming|dp|graph|dijkstra|bfs|dfs)\b",
        r"(?:\b|^)a\*(?:\s|$|\W)"]),
    ("reasoning_comparison", [
        r"\b(compare|contrast|difference between|pros and cons|vs\.?|versus)\b",
        r"\b(evaluate|assess|critique|analyze)\b"]),
    ("long_form_generation", [
        r"\b(essay|report|proposal|research paper|literature review|methodology)\b",
        r"\b(comprehensive|in-depth|step[- ]by[- ]step|detailed)\b",
        r"\b(summarize|synthesis)\b.*\b(everything|all|so far|entire)\b",
        r"\b(transcript|debate|dialogue|format as json|markdown table)\b"]),
    ("data_engineering", [
        r"\b(etl|pipeline|spark|hadoop|presto|sql|csv|excel|dataframe|dataset)\b",
        r"\b(deduplicate|normalize|clean|transform|parse|extract)\b"]),
    ("medical_analysis", [
        r"\b(symptom|diagnosis|treatment|therapy|prognosis|chronic|severe)\b",
        r"\b(pain|migraine|dizziness|fatigue|nausea|inflammation|anxiety|depression)\b",
        r"\b(dietary|meal|training|exercise|recovery)\b.*\b(plan|schedule|regimen)\b",
        r"\b(mental health|psycholog|counseling|therapist|physician|hospital)\b"]),
    ("context_heavy", [
        r"\b(using (all|the) (context|history|above)|based on (the|our) (conversation|context))\b",
        r"\b(continue|expand|build on|follow up)\b.*\b(previous|earlier|above)\b"]),
]

SIMPLE_RULES: List[Tuple[str, List[str]]] = [
    ("greeting", [
        r"\b(hi|hello|hey|yo|sup)\b",
        r"\bgood (morning|afternoon|evening)\b",
        r"\b(thanks|thank you)\b"]),
    ("general_knowledge", [
        r"\b(what is|who is|where is|when is|when did|how many|capital of)\b",
        r"\b(tell me a joke|fun fact|random fact)\b",
        r"\b(how to|how do i|can you tell me)\b"]),
    ("wellness_tips", [
        r"\b(benefits? of|tips? for|advice on)\b",
        r"\b(daily intake|how often|how much)\b",
        r"\b(healthy|good)\b.*\b(habit|routine|lifestyle)\b"]),
    ("short_definition", [
        r"\b(define|meaning of|definition of)\b",
        r"\bwhat does\b.*\bmean\b"]),
    ("tiny_math", [
        r"^\s*\d+\s*[\+\-\*/]\s*\d+\s*\??\s*$",
        r"^\s*what is\s+\d+\s*[\+\-\*/]\s*\d+\s*\??\s*$"]),
]

# Case-sensitive substring markers counted on the raw (stripped) query.
CODE_MARKERS = ("```", "def ", "class ", "import ", "Traceback", "Exception", "ModuleNotFoundError",
                "SELECT ", "WITH ", "FROM ", "JOIN ", ";", "{", "}", "->", "::", "==", "!=")


def _compile(rules: List[Tuple[str, List[str]]]) -> List[Tuple[str, "re.Pattern[str]"]]:
    # One alternation per category: a single regex scan instead of N searches.
    return [(cat, re.compile("|".join(f"(?:{p})" for p in pats), re.IGNORECASE)) for cat, pats in rules]


_COMPLEX = _compile(COMPLEX_RULES)
_SIMPLE = _compile(SIMPLE_RULES)


class HeuristicRouter(BaseRouter):
    name = "heuristic"

    def __init__(self, config: Dict[str, Any]):
        super().__init__(config)
        self.long_text_threshold = int(config.get("heuristic_long_chars", 250))
        self.multi_question_threshold = int(config.get("heuristic_multi_qmarks", 3))
        self.code_markers_needed = int(config.get("heuristic_code_markers_needed", 2))
        self.context_chars_threshold = int(config.get("heuristic_context_chars", 800))
        self._token_fallback = TokenBasedRouter(config)

    @staticmethod
    def _category(text_lower: str, table) -> Optional[str]:
        for cat, rx in table:
            if rx.search(text_lower):
                return cat
        return None

    def route(self, query: str, context: Optional[str] = None) -> RoutingDecision:
        q = (query or "").strip()
        ql = q.lower()

        cat = self._category(ql, _COMPLEX)
        if cat is not None:
            return RoutingDecision(LARGE, 0.92, "heuristic", f"complex pattern={cat}")
        if len(q) >= self.long_text_threshold:
            return RoutingDecision(LARGE, 0.80, "heuristic", f"long query chars={len(q)}")
        nq = q.count("?")
        if nq >= self.multi_question_threshold:
            return RoutingDecision(LARGE, 0.80, "heuristic", f"multi-question count={nq}")
        if sum(1 for m in CODE_MARKERS if m in q) >= self.code_markers_needed:
            return RoutingDecision(LARGE, 0.88, "heuristic", "code/debug markers detected")
        if context and len(context) >= self.context_chars_threshold:
            return RoutingDecision(LARGE, 0.75, "heuristic", f"large context chars={len(context)}")
        scat = self._category(ql, _SIMPLE)
        if scat is not None:
            return RoutingDecision(SMALL, 0.90, "heuristic", f"simple pattern={scat}")
        if len(ql.split()) <= 15 and len(q) <= 100:
            return RoutingDecision(SMALL, 0.75, "heuristic", "short everyday query")
        d = self._token_fallback.route(query, context)
        return RoutingDecision(d.device, float(d.confidence * 0.5), "heuristic_fallback",
                               f"no heuristic match -> {d.reasoning}", d.complexity_score)


# ----------------------------------------------------------------------------- hybrid

def semantic_available(config: Dict[str, Any]) -> bool:
    """Semantic sub-router is available unless explicitly disabled (``"semantic_enabled": False``).

    The reference drops it when sentence-transformers is missing
    (``query_router_engine.py:378``); set ``semantic_enabled=False`` (or env
    ``DLLM_NO_SEMANTIC=1``) to reproduce that probe setup (SURVEY §2.9 golden outputs).
    """
    if os.environ.get("DLLM_NO_SEMANTIC") == "1":
        return False
    return bool(config.get("semantic_enabled", True))


class HybridRouter(BaseRouter):
    name = "hybrid"

    def __init__(self, config: Dict[str, Any]):
        super().__init__(config)
        self.weights = config.get("weights", {"token": 0.35, "semantic": 0.35, "heuristic": 0.30})
        self.routers: Dict[str, Optional[BaseRouter]] = {
            "token": TokenBasedRouter(config),
            "semantic": SemanticRouter(config) if semantic_available(config) else None,
            "heuristic": HeuristicRouter(config),
        }

    def route(self, query: str, context: Optional[str] = None) -> RoutingDecision:
        score = {SMALL: 0.0, LARGE: 0.0}
        parts: List[str] = []
        for name, r in self.routers.items():
            if r is None:
                continue
            d = r.route(query, context)
            w = float(self.weights.get(name, 0.0))
            score[LARGE if d.device == LARGE else SMALL] += w * float(d.confidence)
            parts.append(f"{name}:{d.device} conf={d.confidence:.2f} w={w:.2f}")
        n, o = score[SMALL], score[LARGE]
        final, margin = (LARGE, o - n) if o > n else (SMALL, n - o)
        total = n + o
        conf = margin / total if total > 1e-12 else 0.5
        return RoutingDecision(
            device=final, confidence=float(min(max(conf, 0.0), 1.0)), method="hybrid",
            reasoning=f"nano_score={n:.3f} orin_score={o:.3f} | " + " | ".join(parts))


# ----------------------------------------------------------------------------- perf

class PerformanceAwareRouter(BaseRouter):
    """Sliding-window latency/token + failure-rate scoring (lower wins).

    Running sums make ``score`` O(1) per call; semantics equal the reference's
    recomputation over the deque (``query_router_engine.py:435-445``).
    """
    name = "perf"

    def __init__(self, config: Dict[str, Any]):
        super().__init__(config)
        self.window = int(config.get("perf_window", 30))
        self.fail_penalty = float(config.get("perf_fail_penalty", 3000.0))
        # reference quirk 3: a device without stats scores inf and is never tried
        # once the other has stats; ``perf_explore`` sends the next request to it instead
        self.explore = bool(config.get("perf_explore", False))
        self.stats: Dict[str, deque] = {SMALL: deque(), LARGE: deque()}
        self._sums = {SMALL: [0.0, 0, 0], LARGE: [0.0, 0, 0]}
        self._lock = threading.Lock()

    def update(self, device: str, latency_ms: float, tokens: int, ok: bool = True) -> None:
        if device not in self.stats:
            return
        rec = (float(latency_ms), int(tokens), 1 if ok else 0)
        with self._lock:
            q, s = self.stats[device], self._sums[device]
            q.append(rec)
            s[0] += rec[0]; s[1] += rec[1]; s[2] += rec[2]
            if len(q) > self.window:
                old = q.popleft()
                s[0] -= old[0]; s[1] -= old[1]; s[2] -= old[2]

    def _score(self, device: str) -> float:
        with self._lock:
            n = len(self.stats[device])
            lat, tok, ok = self._sums[device]
        if n == 0:
            return float("inf")
        fail_rate = 1.0 - ok / n
        base = lat / n if tok == 0 else lat / tok
        return float(base + self.fail_penalty * fail_rate)

    def snapshot(self) -> Dict[str, Dict[str, float]]:
        return {d: {"n": len(self.stats[d]), "score": self._score(d)} for d in self.stats}

    def route(self, query: str, context: Optional[str] = None) -> RoutingDecision:
        ns, os_ = self._score(SMALL), self._score(LARGE)
        if ns == float("inf") and os_ == float("inf"):
            return RoutingDecision(SMALL, 0.2, "perf", "no perf stats yet -> default nano")
        if self.explore and (ns == float("inf") or os_ == float("inf")):
            dev = SMALL if ns == float("inf") else LARGE
            return RoutingDecision(dev, 0.2, "perf", f"no perf stats for {dev} yet -> exploring {dev}")
        dev = LARGE if os_ < ns else SMALL
        return RoutingDecision(dev, 0.70, "perf", f"scores nano={ns:.2f} orin={os_:.2f} -> {dev}")


STRATEGIES = {
    "token": TokenBasedRouter,
    "semantic": SemanticRouter,
    "heuristic": HeuristicRouter,
    "hybrid": HybridRouter,
    "perf": PerformanceAwareRouter,
}
