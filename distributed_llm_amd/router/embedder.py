"""Sentence embedders for the semantic router and the semantic routing cache.

The reference encodes with ``SentenceTransformer("all-MiniLM-L6-v2")`` on the host
(``src/query_router_engine.py:126,181,511,571``; ``src/cache.py:412``) and loads up to three
copies of it.  Here every consumer shares ONE embedder per
(name, device) through ``get_embedder``.

Two implementations:
  * ``HashEmbedder`` — deterministic signed feature hashing of word unigrams/bigrams and
    character trigrams into 384 dims, L2-normalised.  No weights needed; lexical overlap
    gives meaningful cosine similarities, so it is the default for CPU runs and tests.
  * ``MiniLMEmbedder`` — the MiniLM-L6 encoder architecture (6 layers, H=384, 12 heads,
    mean-pool + L2) executed on the GPU by ``models.minilm`` entirely on our HIP kernels
    (embedding+LN, bias/GELU/residual GEMM epilogues, encoder attention, LayerNorm, pooling).  Loads real weights from a safetensors file when
    ``DLLM_MINILM_WEIGHTS`` points at one, else random-init with a fixed seed (timing-realistic,
    semantically meaningless — say so when quoting semantic accuracy).
"""
from __future__ import annotations

import hashlib
import os
import re
import threading
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

EMBED_DIM = 384
_WORD_RE = re.compile(r"[a-z0-9]+(?:'[a-z]+)?")


def _h64(s: str) -> int:
    return int.from_bytes(hashlib.blake2b(s.encode("utf-8"), digest_size=8).digest(), "little")


class Embedder:
    dim: int = EMBED_DIM
    name: str = "base"

    def encode(self, texts: Sequence[str]) -> np.ndarray:  # [n, dim] float32
        raise NotImplementedError

    def encode_one(self, text: str) -> np.ndarray:
        return self.encode([text])[0]


class HashEmbedder(Embedder):
    name = "hash"

    def __init__(self, dim: int = EMBED_DIM):
        self.dim = dim
        self._memo: Dict[str, np.ndarray] = {}
        self._lock = threading.Lock()

    def _features(self, text: str) -> List[Tuple[str, float]]:
        t = (text or "").lower()
        words = _WORD_RE.findall(t)
        feats: List[Tuple[str, float]] = [("w:" + w, 1.0) for w in words]
        feats += [("b:" + a + "_" + b, 0.7) for a, b in zip(words, words[1:])]
        squashed = " " + " ".join(words) + " "
        feats += [("c:" + squashed[i:i + 3], 0.35) for i in range(len(squashed) - 2)]
        return feats

    def _one(self, text: str) -> np.ndarray:
        with self._lock:
            hit = self._memo.get(text)
        if hit is not None:
            return hit
        v = np.zeros(self.dim, dtype=np.float32)
        for f, w in self._features(text):
            h = _h64(f)
            v[h % self.dim] += w if (h >> 63) & 1 else -w
        n = float(np.linalg.norm(v))
        if n > 1e-9:
            v /= n
        with self._lock:
            if len(self._memo) > 50000:
                self._memo.clear()
            self._memo[text] = v
        return v

    def encode(self, texts: Sequence[str]) -> np.ndarray:
        if not len(texts):
            return np.zeros((0, self.dim), dtype=np.float32)
        return np.stack([self._one(t) for t in texts])


class MiniLMEmbedder(Embedder):
    """GPU MiniLM-L6 encoder (see ``models.minilm``)."""

    name = "minilm"

    def __init__(self, device: str = "cuda", weights: Optional[str] = None, max_len: int = 256):
        import torch
        from ..models.minilm import MiniLMEncoder, MiniLMConfig
        self.torch = torch
        self.device = torch.device(device)
        cfg = MiniLMConfig(max_position=max(max_len, 512))
        self.model = MiniLMEncoder(cfg, device=self.device)
        weights = weights or os.environ.get("DLLM_MINILM_WEIGHTS")
        if weights and os.path.exists(weights):
            self.model.load_safetensors(weights)
        self.max_len = max_len
        self.dim = cfg.hidden

    def prefetch(self, texts: Sequence[str]) -> None:
        """Encode a routing batch in one forward; its lookups reuse the result (memo or not)."""
        self.model.prefetch(list(texts), max_len=self.max_len)

    def encode_tensor(self, texts: Sequence[str]):
        """Return a [n, dim] float32 device tensor (stays in HBM for the GPU scorer)."""
        return self.model.encode(list(texts), max_len=self.max_len)

    def encode_rows(self, texts: Sequence[str]):
        """One [dim] f32 device row per text (no stacking launch; memo rows are shared)."""
        return self.model.encode_rows(list(texts), max_len=self.max_len)

    def encode(self, texts: Sequence[str]) -> np.ndarray:
        if not len(texts):
            return np.zeros((0, self.dim), dtype=np.float32)
        return self.encode_tensor(texts).float().cpu().numpy()


_REGISTRY: Dict[Tuple[str, str], Embedder] = {}
_REG_LOCK = threading.Lock()


def resolve_embedder_kind(model_name: str) -> str:
    """Map a config ``embedding_model`` to an implementation.

    ``DLLM_EMBEDDER`` (hash|minilm) overrides; otherwise MiniLM names select the GPU
    encoder only when a GPU is present, else the hash embedder.
    """
    env = os.environ.get("DLLM_EMBEDDER")
    if env:
        return env
    if model_name and model_name.lower() in ("hash", "hash-384"):
        return "hash"
    try:
        import torch
        if torch.cuda.is_available() and "minilm" in (model_name or "").lower():
            return "minilm"
    except Exception:
        pass
    return "hash"


def get_embedder(model_name: str = "all-MiniLM-L6-v2", device: Optional[str] = None) -> Embedder:
    kind = resolve_embedder_kind(model_name)
    dev = device or ("cuda" if kind == "minilm" else "cpu")
    key = (kind, dev)
    with _REG_LOCK:
        emb = _REGISTRY.get(key)
        if emb is None:
            emb = MiniLMEmbedder(device=dev) if kind == "minilm" else HashEmbedder()
            _REGISTRY[key] = emb
    return emb


def encoder_stats() -> Dict[str, float]:
    """Summed per-text memo counters of the GPU encoders in the registry (hash embedders have no
    kernels to report): lookups, hits, texts actually run through the encoder."""
    tot = {"lookups": 0, "hits": 0, "encoded_texts": 0, "batch_hits": 0}
    kinds = []
    with _REG_LOCK:
        embs = list(_REGISTRY.values())
    for e in embs:
        kinds.append(e.name)
        if isinstance(e, MiniLMEmbedder):
            st = e.model.memo_stats()
            for k in tot:
                tot[k] += st[k]
            tot["memo_enabled"] = st["memo_enabled"]
    tot["kinds"] = sorted(set(kinds))
    return tot


def clear_registry() -> None:
    with _REG_LOCK:
        _REGISTRY.clear()
