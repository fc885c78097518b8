"""QueryRouter: strategy selector in front of the predictive routing cache.

Reference: ``src/query_router_engine.py:465-691`` (registry :478-484, ctor :486-511,
``route_query`` :559-645, cache helpers :651-677, ``update_perf`` :683-685,
``change_strategy`` :687-691).

Cache-hit policy (identical to the reference):
  * context ≥ ``heuristic_context_chars`` (default 800) and cached prediction is the small
    tier, or prediction confidence below ``prediction_confidence_threshold``
    → re-route with the *current* strategy, record the decision, mark ``cache_hit``;
  * otherwise return the predicted tier with method ``"<strategy>_cached"``.

Fixes kept behind flags:
  * ``change_strategy`` keeps perf statistics when switching *to* perf and back
    (``"preserve_perf_on_switch"``, default True — the reference discards them, quirk 4).
"""
from __future__ import annotations

import logging
import threading
from datetime import datetime
from typing import Any, Dict, List, Optional, Tuple

from ..config import SMALL, resolve_config
from .cache import QueryCache
from .embedder import get_embedder
from .strategies import STRATEGIES, PerformanceAwareRouter, RoutingDecision

logger = logging.getLogger(__name__)


class QueryRouter:
    AVAILABLE_STRATEGIES = STRATEGIES

    def __init__(self, strategy: str = "token", config: Optional[Dict[str, Any]] = None):
        self.config = resolve_config(config)
        if strategy not in self.AVAILABLE_STRATEGIES:
            raise ValueError(f"Unknown strategy={strategy}. Available={list(self.AVAILABLE_STRATEGIES)}")
        self._lock = threading.RLock()
        self._perf_router: Optional[PerformanceAwareRouter] = None
        self.strategy_name = strategy
        self.router = self._build(strategy)
        self.cache_enabled = bool(self.config.get("cache_enabled", True))
        index_device = self.config.get("cache_index_device")
        self._cache = QueryCache(
            max_size=int(self.config.get("cache_max_size", 500)),
            ttl_seconds=int(self.config.get("cache_ttl_seconds", 3600)),
            similarity_threshold=float(self.config.get("cache_similarity_threshold", 0.85)),
            use_semantic=bool(self.config.get("use_semantic_cache", True)),
            prediction_confidence_threshold=float(self.config.get("prediction_confidence_threshold", 0.70)),
            index_device=index_device,
        )
        self.cache_embedder = None
        if self.config.get("use_semantic_cache", True):
            self.cache_embedder = get_embedder(self.config.get("embedding_model", "all-MiniLM-L6-v2"))

    def _build(self, strategy: str):
        if strategy == "perf" and self.config.get("preserve_perf_on_switch", True):
            if self._perf_router is None:
                self._perf_router = PerformanceAwareRouter(self.config)
            return self._perf_router
        return self.AVAILABLE_STRATEGIES[strategy](self.config)

    @property
    def strategy(self) -> str:
        return self.strategy_name

    def _embed(self, query: str):
        rows = getattr(self.cache_embedder, "encode_rows", None)
        if rows is not None and self.config.get("cache_index_device"):
            return rows([query])[0]
        return self.cache_embedder.encode([query])[0]

    def prefetch_cache(self, queries: List[str], context_keys: List[Optional[str]]) -> None:
        """Score a routing batch's semantic-cache lookups together (QueryCache.prefetch: one GPU
        launch + one read-back on an HBM index); ``route_query`` then consumes them in order."""
        if not (self.cache_enabled and self.cache_embedder is not None and queries):
            return
        try:
            items = [(q, ck or "default", self._embed(q)) for q, ck in zip(queries, context_keys)]
        except Exception as exc:  # noqa: BLE001 - route_query retries per query and logs
            logger.debug("cache prefetch skipped: %s", exc)
            return
        self._cache.prefetch(items)

    def prefetch_scores(self, queries: List[str]) -> None:
        """Batch the semantic centroid scoring of a routing batch (SemanticRouter.prefetch), for
        the semantic strategy and the semantic member of the hybrid one."""
        from .strategies import SemanticRouter
        r = self.router
        for x in [r] + list((getattr(r, "routers", None) or {}).values()):
            if isinstance(x, SemanticRouter):
                x.prefetch(queries)

    def route_query(self, query: str, context: Optional[str] = None,
                    context_key: Optional[str] = None) -> RoutingDecision:
        ctxk = context_key or "default"
        q_emb = None
        if self.cache_enabled and self.cache_embedder is not None:
            try:
                q_emb = self._embed(query)
            except Exception as exc:  # the reference continues without an embedding
                logger.warning("Cache embedding failed, continuing without: %s", exc)

        if self.cache_enabled:
            hit = self._cache.lookup(query, ctxk, q_emb)
            if hit is not None:
                ctx_len = len(context) if context else 0
                ctx_thr = int(self.config.get("heuristic_context_chars", 800))
                override = ctx_len >= ctx_thr and hit.predicted_device == SMALL
                if override or hit.use_hybrid_fallback:
                    reason = (f"context_len={ctx_len}>={ctx_thr} overrides cached nano" if override
                              else f"low prediction confidence={hit.predicted_confidence:.2f}")
                    d = self.router.route(query, context)
                    self._cache.insert(query, ctxk, device=d.device, confidence=d.confidence,
                                       method=d.method, q_emb=q_emb)
                    d.reasoning = f"cache hit (hybrid re-route: {reason}) | " + d.reasoning
                    d.cache_hit = True
                    return d
                age = int((datetime.now() - hit.entry.timestamp).total_seconds())
                return RoutingDecision(
                    device=hit.predicted_device, confidence=hit.predicted_confidence,
                    method=f"{self.strategy_name}_cached",
                    reasoning=(f"cache hit age={age}s hits={hit.entry.hit_count} "
                               f"predicted={hit.predicted_device} conf={hit.predicted_confidence:.2f} "
                               f"context_len={ctx_len} history={len(hit.entry.routing_history)}"),
                    cache_hit=True)

        d = self.router.route(query, context)
        if self.cache_enabled:
            self._cache.insert(query, ctxk, device=d.device, confidence=d.confidence,
                               method=d.method, q_emb=q_emb)
        return d

    # -- cache passthroughs (reference :651-677)
    def warm_up_cache(self, pairs: List[Tuple[str, str, str]]) -> None:
        self._cache.warm_up(pairs, embedder=self.cache_embedder)

    def save_cache(self, path: str) -> None:
        self._cache.save(path)

    def load_cache(self, path: str) -> int:
        return self._cache.load(path)

    def invalidate_cache(self, context_key: Optional[str] = None, query_pattern: Optional[str] = None) -> int:
        return self._cache.invalidate(context_key=context_key, query_pattern=query_pattern)

    def get_cache_stats(self) -> Dict[str, Any]:
        return self._cache.stats()

    def clear_cache(self) -> None:
        self._cache.clear()

    # -- perf feedback + hot swap (reference :683-691)
    def update_perf(self, device: str, latency_ms: float, tokens: int, ok: bool = True) -> None:
        upd = getattr(self.router, "update", None)
        if upd is not None:
            upd(device=device, latency_ms=latency_ms, tokens=tokens, ok=ok)
        elif self._perf_router is not None:
            self._perf_router.update(device=device, latency_ms=latency_ms, tokens=tokens, ok=ok)

    def change_strategy(self, strategy: str) -> None:
        if strategy not in self.AVAILABLE_STRATEGIES:
            raise ValueError(f"Unknown strategy={strategy}")
        with self._lock:
            self.router = self._build(strategy)
            self.strategy_name = strategy


def smoke(cache_path: str = "/tmp/qr_cache.json", strategy: str = "hybrid") -> Dict[str, Any]:
    """Routing-engine smoke run (reference query_router_engine.py:734-764): warm the cache with two
    labelled pairs, route three queries, route them again (predictive hits from the routing
    history), print cache statistics and persist the cache as JSON.

    The reference runs this on BENCHMARK_CFG, whose ``cache_enabled`` is False — so its second
    pass never hits; here the cache is switched on so the predictive path is what gets exercised.
    """
    from ..config import BENCHMARK_CFG
    qr = QueryRouter(strategy=strategy, config=dict(BENCHMARK_CFG, cache_enabled=True))
    qr.warm_up_cache([("hello", "demo", "nano"), ("what is 2+2", "demo", "nano")])
    tests = ["hello", "what is 2+2", "Explain quantum computing and its implications for cryptography"]
    first = []
    for t in tests:
        d = qr.route_query(t, context_key="demo")
        first.append(d)
        print(f"{t!r:55} => {d.device:4}  [{d.method}]  {d.reasoning}")
    stats = qr.get_cache_stats()
    print("\nCache stats:", stats)
    print("\n--- Second pass (predictive routing from history) ---")
    second = []
    for t in tests:
        d = qr.route_query(t, context_key="demo")
        second.append(d)
        print(f"{t!r:55} => {d.device:4}  [{d.method}]  cache_hit={d.cache_hit}")
    qr.save_cache(cache_path)
    print(f"\nCache saved to {cache_path}")
    return {"first": first, "second": second, "stats": qr.get_cache_stats()}


if __name__ == "__main__":
    import argparse
    logging.basicConfig(level=logging.INFO)
    _ap = argparse.ArgumentParser()
    _ap.add_argument("--cache-path", default="/tmp/qr_cache.json")
    _ap.add_argument("--strategy", default="hybrid")
    _a = _ap.parse_args()
    smoke(_a.cache_path, _a.strategy)
