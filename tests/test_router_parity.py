"""Routing parity against the reference implementation itself (pure Python, run unmodified
from /root/reference/src when it is mounted; skipped otherwise).

The reference needs sentence-transformers / litellm, which are not installed: litellm is
absent in both implementations (len//4 token fallback), and a stand-in ``SentenceTransformer``
that wraps our deterministic HashEmbedder is injected into the reference module so the
semantic and hybrid strategies are compared on identical embeddings.
"""
import importlib
import os
import sys
import types

import numpy as np
import pytest

REF_SRC = "/root/reference/src"
pytestmark = pytest.mark.skipif(not os.path.isdir(REF_SRC), reason="reference not mounted")

from distributed_llm_amd.bench.query_sets import normalize_query_set, query_sets  # noqa: E402
from distributed_llm_amd.config import BENCHMARK_CFG, PRODUCTION_CFG, DEFAULT_LABEL_PATH  # noqa: E402
from distributed_llm_amd.router.embedder import HashEmbedder  # noqa: E402
from distributed_llm_amd.router.query_router import QueryRouter  # noqa: E402


@pytest.fixture(scope="module")
def refmod():
    sys.path.insert(0, REF_SRC)
    try:
        qre = importlib.import_module("query_router_engine")
    finally:
        sys.path.remove(REF_SRC)
    emb = HashEmbedder()

    class FakeST:
        def __init__(self, name):
            self.name = name

        def encode(self, texts):
            return emb.encode(list(texts))

    qre.SentenceTransformer = FakeST
    qre.SENTENCE_TRANSFORMERS_AVAILABLE = True
    return qre


def _cfg(base, **kw):
    c = dict(base)
    c["semantic_label_path"] = os.path.join(REF_SRC, "tests", "semantic_labels.json")
    c.update(kw)
    return c


def _mine_cfg(base, **kw):
    c = dict(base)
    c["semantic_label_path"] = DEFAULT_LABEL_PATH
    c.update(kw)
    return c


def _conversation(items):
    """(query, context) per turn of a growing conversation with a fixed fake assistant reply."""
    hist = []
    for it in items:
        ctx = "\n".join(f"{r}: {c}" for r, c in hist) or None
        yield it.text, ctx
        hist += [("user", it.text), ("assistant", "Sure. " + it.text[::-1] * 3)]


@pytest.mark.parametrize("strategy", ["token", "heuristic", "semantic", "hybrid"])
@pytest.mark.parametrize("qset", sorted(query_sets))
@pytest.mark.parametrize("thr", [100, 500, 1000, 2000])
def test_strategy_decisions_match_reference(refmod, strategy, qset, thr):
    items = normalize_query_set(query_sets[qset])
    ref = refmod.QueryRouter(strategy, _cfg(BENCHMARK_CFG, token_threshold=thr))
    mine = QueryRouter(strategy, _mine_cfg(BENCHMARK_CFG, token_threshold=thr))
    for q, ctx in _conversation(items):
        a = ref.route_query(q, ctx, "k")
        b = mine.route_query(q, ctx, "k")
        assert (a.device, a.method, a.reasoning) == (b.device, b.method, b.reasoning)
        assert a.confidence == pytest.approx(b.confidence, abs=1e-9)


def test_class_default_thresholds_match(refmod):
    # the live server passes a small dict (replace semantics -> class fallbacks 250/3/800)
    cfg = {"cache_enabled": True, "enable_response_cache": True, "weights": {"token": 0.25, "semantic": 0.45, "heuristic": 0.30}}
    for name in ("heuristic", "hybrid", "token"):
        ref = refmod.QueryRouter(name, dict(cfg))
        mine = QueryRouter(name, dict(cfg))
        for qset in query_sets:
            for q, ctx in _conversation(normalize_query_set(query_sets[qset])):
                a, b = ref.route_query(q, ctx, "c"), mine.route_query(q, ctx, "c")
                assert (a.device, a.method, a.cache_hit) == (b.device, b.method, b.cache_hit), q


def test_perf_router_matches(refmod):
    ref = refmod.QueryRouter("perf", _cfg(BENCHMARK_CFG))
    mine = QueryRouter("perf", _mine_cfg(BENCHMARK_CFG))
    rng = np.random.default_rng(0)
    for i in range(80):
        a, b = ref.route_query("q", None, "k"), mine.route_query("q", None, "k")
        assert (a.device, a.reasoning, a.confidence) == (b.device, b.reasoning, b.confidence)
        dev = ["nano", "orin"][int(rng.integers(0, 2))]
        lat, tok, ok = float(rng.uniform(10, 5000)), int(rng.integers(0, 400)), bool(rng.random() > 0.2)
        ref.update_perf(dev, lat, tok, ok)
        mine.update_perf(dev, lat, tok, ok)


@pytest.mark.parametrize("strategy", ["heuristic", "hybrid", "semantic"])
def test_predictive_cache_matches_reference(refmod, strategy):
    """Production config: exact + semantic hits, context override, low-confidence re-route."""
    ref = refmod.QueryRouter(strategy, _cfg(PRODUCTION_CFG))
    mine = QueryRouter(strategy, _mine_cfg(PRODUCTION_CFG))
    script = [("hello", None, "a"), ("hello", None, "a"), ("Hello!", None, "a"), ("hello", "x" * 4000, "a"),
              ("hello", None, "b"), ("Write a Python function for knapsack", None, "a"),
              ("write a python function for knapsack", None, "a"), ("Thank you!", None, "a"),
              ("thank you", None, "a"), ("hello", None, "a")]
    for q, ctx, key in script:
        a, b = ref.route_query(q, ctx, key), mine.route_query(q, ctx, key)
        assert (a.device, a.method, a.cache_hit) == (b.device, b.method, b.cache_hit), q
        assert a.confidence == pytest.approx(b.confidence, abs=1e-9), q
        # reasoning may embed the entry age in seconds; compare with the age stripped
        strip = lambda s: " ".join(w for w in s.split() if not w.startswith("age="))
        assert strip(a.reasoning) == strip(b.reasoning), q
    sa, sb = ref.get_cache_stats(), mine.get_cache_stats()
    for k in ("size", "valid", "stale", "hits", "attempts", "hit_rate", "evictions", "hybrid_fallbacks"):
        assert sa[k] == sb[k], k
    assert sa["top_queries"] == sb["top_queries"]


def test_cache_prediction_and_persistence(refmod, tmp_path):
    cache_mod = sys.modules["cache"]
    from distributed_llm_amd.router.cache import QueryCache
    ref, mine = cache_mod.QueryCache(max_size=3, ttl_seconds=100), QueryCache(max_size=3, ttl_seconds=100)
    seq = [("a", "k", "nano", 0.9), ("a", "k", "orin", 0.9), ("b", "k", "orin", 0.4), ("c", "k", "nano", 1.0),
           ("d", "k", "nano", 1.0), ("a", "k", "orin", 0.2)]
    for q, k, d, c in seq:
        ref.insert(q, k, d, c, "m")
        mine.insert(q, k, d, c, "m")
    for q in ("a", "b", "c", "d", "zzz"):
        ra, rb = ref.lookup(q, "k"), mine.lookup(q, "k")
        assert (ra is None) == (rb is None)
        if ra:
            assert (ra.predicted_device, ra.use_hybrid_fallback) == (rb.predicted_device, rb.use_hybrid_fallback)
            assert ra.predicted_confidence == pytest.approx(rb.predicted_confidence)
    p1, p2 = tmp_path / "r.json", tmp_path / "m.json"
    ref.save(str(p1))
    mine.save(str(p2))
    # file formats are interchangeable
    assert QueryCache(ttl_seconds=100).load(str(p1)) == cache_mod.QueryCache(ttl_seconds=100).load(str(p2)) == 3


def test_cache_ttl_expiry_parity(refmod):
    """TTL eviction (reference cache.py:250,523-538): entries older than ttl are evicted on lookup
    and preferred as the victim when full; refreshed entries survive.  Ours uses an expiry heap."""
    import time
    cache_mod = sys.modules["cache"]
    from distributed_llm_amd.router.cache import QueryCache
    ref, mine = cache_mod.QueryCache(max_size=3, ttl_seconds=0.3), QueryCache(max_size=3, ttl_seconds=0.3)
    for c in (ref, mine):
        c.insert("a", "k", "nano", 0.9, "m")
        c.insert("b", "k", "orin", 0.9, "m")
    time.sleep(0.2)
    for c in (ref, mine):
        c.insert("b", "k", "orin", 0.8, "m")      # refresh b
        c.insert("c", "k", "nano", 0.8, "m")
    time.sleep(0.15)                               # a expired, b and c alive
    for c in (ref, mine):
        c.insert("d", "k", "orin", 0.7, "m")      # full: the stale entry (a) is the victim
    for q in ("a", "b", "c", "d"):
        assert (ref.lookup(q, "k") is None) == (mine.lookup(q, "k") is None), q
    sa, sb = ref.stats(), mine.stats()
    for k in ("size", "valid", "stale", "hits", "attempts", "evictions"):
        assert sa[k] == sb[k], k
    time.sleep(0.35)                               # everything expires
    assert ref.lookup("d", "k") is None and mine.lookup("d", "k") is None
    assert ref.stats()["size"] == mine.stats()["size"] == 0
    assert ref.stats()["evictions"] == mine.stats()["evictions"]


def test_router_smoke_entry(tmp_path, monkeypatch):
    """Routing-engine smoke (reference query_router_engine.py:734-764): warm-up, two passes, save."""
    import json as _json
    monkeypatch.setenv("DLLM_EMBEDDER", "hash")
    from distributed_llm_amd.router.embedder import clear_registry
    from distributed_llm_amd.router.query_router import smoke
    clear_registry()
    path = str(tmp_path / "qr_cache.json")
    res = smoke(path)
    assert [d.device for d in res["first"][:2]] == ["nano", "nano"]
    assert all(d.cache_hit for d in res["second"])
    with open(path) as f:
        entries = _json.load(f)
    assert {e["query"] for e in entries} >= {"hello", "what is 2+2"}
    clear_registry()
