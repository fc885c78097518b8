"""Batched semantic-cache lookups (QueryCache.prefetch) must route exactly like per-query lookups.

The reference scores every lookup on its own against the entries of the same context_key
(src/cache.py:267-305).  Here a routing batch is scored at once (one GPU launch on an HBM index);
a prefetched result is used only while no row of its context changed since the batch was scored.
This workload makes such changes happen inside batches on purpose: queries of one batch that share
a context (an insert of one must be seen by a later one), near-duplicate queries (semantic hits),
replacements, LRU evictions (a small max_size) - and compares every decision with a cache that
never prefetches.  Runs on the host numpy index here and on the HBM index in test_router_gpu.py.
"""
import numpy as np
import pytest

from distributed_llm_amd.router.cache import QueryCache


def _workload(seed=0, batches=40, B=24, dim=32, n_ctx=6):
    rng = np.random.default_rng(seed)
    base = rng.standard_normal((60, dim)).astype(np.float32)
    out = []
    for b in range(batches):
        items = []
        for i in range(B):
            k = int(rng.integers(0, 60))
            ctx = f"ctx{int(rng.integers(0, n_ctx))}" if rng.random() < 0.8 else f"uniq{b}_{i}"
            v = base[k] + (0.15 * rng.standard_normal(dim)).astype(np.float32)
            q = f"query {k}" if rng.random() < 0.5 else f"query {k} v{int(rng.integers(0, 4))}"
            items.append((q, ctx, v))
        out.append(items)
    return out


def _run(cache: QueryCache, batches, prefetch: bool, to_dev=None):
    trace = []
    for items in batches:
        if to_dev is not None:
            items = [(q, c, to_dev(v)) for q, c, v in items]
        if prefetch:
            cache.prefetch(items)
        for j, (q, c, v) in enumerate(items):
            hit = cache.lookup(q, c, v)
            if hit is None:
                cache.insert(q, c, "nano" if j % 3 else "orin", 0.8, "token", q_emb=v)
                trace.append(("miss", q, c))
            else:
                trace.append(("hit", hit.entry.query, hit.predicted_device, round(hit.predicted_confidence, 6)))
                if hit.use_hybrid_fallback or j % 5 == 0:   # re-route on a hit: records + replaces the row
                    cache.insert(q, c, "orin", 0.9, "hybrid", q_emb=v)
    return trace


@pytest.mark.parametrize("max_size", [500, 40])
def test_prefetched_lookups_equal_per_query_lookups(max_size):
    batches = _workload()
    a = QueryCache(max_size=max_size, ttl_seconds=3600, similarity_threshold=0.9, dim=32)
    b = QueryCache(max_size=max_size, ttl_seconds=3600, similarity_threshold=0.9, dim=32)
    ta, tb = _run(a, batches, True), _run(b, batches, False)
    assert ta == tb
    assert sum(1 for t in ta if t[0] == "hit") > 30          # semantic + exact hits happened
    assert a.prefetch_used > 100 and a.prefetch_fallbacks > 0  # both paths exercised
    sa, sb = a.stats(), b.stats()
    for k in ("size", "hits", "attempts", "evictions", "hybrid_fallbacks"):
        assert sa[k] == sb[k], k


def test_prefetch_tracking_is_off_without_a_batch():
    c = QueryCache(max_size=50, ttl_seconds=3600, similarity_threshold=0.9, dim=8)
    v = np.ones(8, dtype=np.float32)
    for i in range(20):
        c.insert(f"q{i}", f"c{i}", "nano", q_emb=v)
    assert not c._index.dirty and not c._index.track_dirty
    c.prefetch([("q1", "c1", v)])
    assert c._index.track_dirty
    assert c.lookup("q1", "c1", v) is not None
    assert not c._index.track_dirty      # the batch was consumed
