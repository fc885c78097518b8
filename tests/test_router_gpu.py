"""Router components on the GPU: the HBM embedding index fed with device embeddings (no host round
trip per insert) against the host numpy index, batched semantic centroid scoring against the
per-query path through the whole orchestrator, and cache snapshots holding device embeddings."""
import os

import numpy as np
import pytest
import torch

from distributed_llm_amd.router.cache import EmbeddingIndex, QueryCache

pytestmark = pytest.mark.gpu


def test_device_index_matches_host_index():
    rng = np.random.default_rng(0)
    host, dev = EmbeddingIndex(dim=64, capacity=8), EmbeddingIndex(dim=64, capacity=8, device="cuda")
    vecs = rng.standard_normal((40, 64)).astype(np.float32)
    ctxs = [f"c{i % 3}" for i in range(40)]
    for i, (v, c) in enumerate(zip(vecs, ctxs)):   # grows twice; half the rows arrive as device tensors
        host.put(v, c)
        dev.put(torch.from_numpy(v).cuda() if i % 2 else v, c)
    for i in (3, 17, 30):                           # replacement + removal keep both in step
        host.remove(i)
        dev.remove(i)
    host.put(vecs[5] * 2.0, "c1", slot=7)
    dev.put(torch.from_numpy(vecs[5] * 2.0).cuda(), "c1", slot=7)
    for j in range(12):
        q = vecs[j] + 0.05 * rng.standard_normal(64).astype(np.float32)
        for c in ("c0", "c1", "c2", "nope"):
            hs, hv = host.best(q, c, 0.5)
            ds, dv = dev.best(torch.from_numpy(q).cuda(), c, 0.5)
            assert hs == ds, (j, c, hs, ds)
            assert abs(hv - dv) < 1e-4


def test_cache_with_device_embeddings_round_trips(tmp_path):
    c = QueryCache(max_size=64, index_device="cuda", dim=32)
    rng = np.random.default_rng(1)
    embs = torch.from_numpy(rng.standard_normal((5, 32)).astype(np.float32)).cuda()
    for i in range(5):
        c.insert(f"query {i}", "ctx", device="orin" if i % 2 else "nano", confidence=0.9, method="m", q_emb=embs[i])
    hit = c.lookup("something else", "ctx", embs[3] * 1.01)
    assert hit is not None and hit.entry.query == "query 3"
    c.save_snapshot(tmp_path / "snap.safetensors")
    c.save(str(tmp_path / "cache.json"))
    for loader in ("load_snapshot", "load"):
        d = QueryCache(max_size=64, index_device="cuda", dim=32)
        path = tmp_path / ("snap.safetensors" if loader == "load_snapshot" else "cache.json")
        assert getattr(d, loader)(str(path)) == 5
        hit = d.lookup("x", "ctx", embs[2])
        assert hit is not None and hit.entry.query == "query 2"


def test_batched_semantic_scores_match_per_query(monkeypatch):
    """route_batch with the batched centroid scores == the same batch routed with the per-query
    scorer (hybrid strategy, GPU MiniLM encoder, HBM routing cache)."""
    from distributed_llm_amd.config import LARGE, PRODUCTION_CFG, SMALL
    from distributed_llm_amd.orchestrator import Router
    from distributed_llm_amd.pools.base import EchoPool
    from distributed_llm_amd.router.strategies import SemanticRouter
    monkeypatch.setenv("DLLM_EMBEDDER", "minilm")
    cfg = dict(PRODUCTION_CFG, cache_index_device="cuda", enable_response_cache=False)
    hist = [[{"role": "user", "content": f"[s{i}] " + q}] for i, q in enumerate(
        ["what is the capital of france", "write a python function to reverse a linked list",
         "explain the difference between tcp and udp in detail", "hi", "prove that sqrt 2 is irrational",
         "how do I fix a segfault in my C code", "tell me a joke", "compare quicksort and mergesort"] * 3)]

    def run(batched: bool):
        if not batched:
            monkeypatch.setattr(SemanticRouter, "prefetch", lambda self, qs: None)
        r = Router(strategy="hybrid", config=cfg, pools={SMALL: EchoPool(SMALL), LARGE: EchoPool(LARGE)})
        out = [(p["routing_method"], p["routing_confidence"], dev) for p, _, dev in r.route_batch(hist)]
        monkeypatch.undo()
        monkeypatch.setenv("DLLM_EMBEDDER", "minilm")
        return out

    assert run(True) == run(False)


def test_cache_scan_matches_fp32_reference():
    """The batched scorer (one launch per 128 queries) against the fp32 torch reference: several
    queries per context, more than 128 queries, a row count that is not a multiple of 4, zero rows,
    removed rows (ctx -1) and a context with no rows."""
    from distributed_llm_amd import ops
    from distributed_llm_amd.ops import reference as ref
    g = torch.Generator(device="cpu").manual_seed(3)
    n, d = 4099, 384
    table = torch.randn(n, d, generator=g).cuda()
    ctx = torch.randint(0, 37, (n,), generator=g, dtype=torch.int32).cuda()
    table[5] = 0.0
    ctx[7:20] = -1
    base = [int(x) for x in torch.randint(0, n, (150,), generator=g)]
    qs = [(table[i] + 0.3 * torch.randn(d, generator=g).cuda()).contiguous() for i in base]
    qs[3] = torch.zeros(d, device="cuda")
    cids = [int(ctx[i]) if int(ctx[i]) >= 0 else 99 for i in base]
    cids[10] = 1000   # no such context
    got = ops.cache_scan(qs, cids, table, ctx, n, 0.7)
    want = ref.cache_scan(qs, cids, table, ctx, n, 0.7)
    hits = 0
    for (gs, gv), (ws, wv) in zip(got, want):
        assert gs == ws, (gs, ws, gv, wv)
        assert abs(gv - wv) < 1e-4
        hits += gs >= 0
    assert hits > 100
    # only the first rows: n_rows bounds the scan
    got = ops.cache_scan(qs[:20], cids[:20], table, ctx, 1000, 0.7)
    assert got == [(s, v) if s < 1000 else (-1, 0.0) for s, v in got]
    assert [s for s, _ in got] == [s for s, _ in ref.cache_scan(qs[:20], cids[:20], table, ctx, 1000, 0.7)]


def test_cache_write_applies_rows_and_removals():
    from distributed_llm_amd import ops
    table = torch.zeros(300, 64, device="cuda")
    ctx = torch.full((300,), -1, dtype=torch.int32, device="cuda")
    vecs = [torch.randn(64, device="cuda") for _ in range(100)]
    ops.cache_write([(i * 3, v, i % 5) for i, v in enumerate(vecs)], table, ctx)   # two launches
    for i, v in enumerate(vecs):
        assert torch.equal(table[i * 3], v) and int(ctx[i * 3]) == i % 5
    ops.cache_write([(0, None, -1), (3, None, 7)], table, ctx)
    assert int(ctx[0]) == -1 and int(ctx[3]) == 7 and torch.equal(table[3], vecs[1])


def test_device_prefetch_equals_per_query_and_batches_launches():
    """The HBM index through QueryCache.prefetch routes exactly like per-query lookups (the CPU
    version of this workload: tests/test_cache_prefetch.py) and issues one scoring launch per
    batch plus one write launch per 64 inserts, instead of a launch (and a read-back) per lookup."""
    import importlib.util
    import pathlib
    spec = importlib.util.spec_from_file_location(
        "tcp", pathlib.Path(__file__).with_name("test_cache_prefetch.py"))
    tcp = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(tcp)
    batches = tcp._workload(seed=1)
    to_dev = lambda v: torch.from_numpy(v).cuda()
    a = QueryCache(max_size=40, ttl_seconds=3600, similarity_threshold=0.9, dim=32, index_device="cuda")
    b = QueryCache(max_size=40, ttl_seconds=3600, similarity_threshold=0.9, dim=32, index_device="cuda")
    h = QueryCache(max_size=40, ttl_seconds=3600, similarity_threshold=0.9, dim=32)
    ta = tcp._run(a, batches, True, to_dev)
    tb = tcp._run(b, batches, False, to_dev)
    th = tcp._run(h, batches, False)
    assert ta == tb == th
    la = a._index.launches
    assert a.prefetch_used > 100
    # per batch: one prefetch scan, plus one per fallback lookup; writes batched per flush
    assert la["scan"] <= len(batches) + a.prefetch_fallbacks + 1
    assert la["scan"] < b._index.launches["scan"]
