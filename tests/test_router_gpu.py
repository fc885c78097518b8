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
