"""Thread-safety stress: the reference mutates `_attempts` outside its cache lock
(`src/cache.py:249`) and leaves the perf deques (`query_router_engine.py:426-429`), the response
store (`router.py:59`) and the Flask globals (`app.py:17-24`) unsynchronised. These tests hammer
our equivalents from many threads and check that the counters and structures stay exact."""
import threading

import numpy as np

from distributed_llm_amd.config import LARGE, PRODUCTION_CFG, SMALL
from distributed_llm_amd.orchestrator import Router
from distributed_llm_amd.pools.base import EchoPool
from distributed_llm_amd.router.cache import QueryCache
from distributed_llm_amd.router.strategies import PerformanceAwareRouter

T = 8


def run_threads(fn, n=T):
    errs = []
    start = threading.Barrier(n)

    def wrap(i):
        try:
            start.wait()
            fn(i)
        except Exception as exc:  # surfaced below
            errs.append(repr(exc))

    ts = [threading.Thread(target=wrap, args=(i,)) for i in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not errs, errs[:3]


def test_query_cache_counters_exact_under_contention():
    cache = QueryCache(max_size=64, ttl_seconds=300, similarity_threshold=0.9, use_semantic=True, dim=16)
    per = 400
    rng = np.random.default_rng(0)
    embs = rng.standard_normal((32, 16)).astype(np.float32)
    embs /= np.linalg.norm(embs, axis=1, keepdims=True)

    def work(i):
        for j in range(per):
            k = (i * 7 + j) % 32
            q = f"query {k}"
            ctx = f"ctx{k % 4}"
            if j % 3 == 0:
                cache.insert(q, ctx, SMALL if k % 2 else LARGE, 0.9, "t", q_emb=embs[k])
            cache.lookup(q, ctx, q_emb=embs[k])
            if j % 50 == 0:
                cache.stats()
            if j % 97 == 0:
                cache.invalidate(context_key=f"ctx{j % 4}")

    run_threads(work)
    st = cache.stats()
    assert st["attempts"] == T * per            # every lookup counted exactly once
    assert 0 < st["hits"] <= st["attempts"]
    assert st["size"] <= 64 and st["size"] == st["valid"] + st["stale"]


def test_perf_router_window_consistent_under_contention():
    r = PerformanceAwareRouter({"perf_window": 30})

    def work(i):
        for j in range(2000):
            r.update(SMALL if (i + j) % 2 else LARGE, 10.0 + i, 5, ok=(j % 5 != 0))
            if j % 10 == 0:
                r.route("hello")

    run_threads(work)
    for dev in (SMALL, LARGE):
        q = r.stats[dev]
        assert len(q) == 30
        lat, tok, ok = r._sums[dev]
        assert abs(lat - sum(x[0] for x in q)) < 1e-6 and tok == sum(x[1] for x in q)
        assert ok == sum(x[2] for x in q)


def test_router_concurrent_sessions_with_response_cache():
    cfg = dict(PRODUCTION_CFG, enable_response_cache=True)
    pools = {SMALL: EchoPool(SMALL, 8), LARGE: EchoPool(LARGE, 16)}
    router = Router("hybrid", config=cfg, pools=pools)
    per = 60
    results = [[] for _ in range(T)]

    def work(i):
        hist = []
        for j in range(per):
            # half the threads share query texts so the response cache is read and written concurrently
            q = f"what is item {j % 10}?" if i % 2 else f"thread {i} question {j} about databases"
            hist.append({"role": "user", "content": q})
            payload, toks, dev = router.route_query(list(hist))
            assert payload["ok"] and dev in (SMALL, LARGE)
            hist.append({"role": "assistant", "content": payload["response"]})
            results[i].append(payload["cache_hit"])

    run_threads(work)
    assert sum(len(r) for r in results) == T * per
    assert pools[SMALL].calls + pools[LARGE].calls <= T * per
    st = router.query_router.get_cache_stats()
    assert st["attempts"] >= 1 and st["hits"] <= st["attempts"]


def test_http_api_concurrent_sessions():
    from distributed_llm_amd.server.app import create_app
    pools = {SMALL: EchoPool(SMALL, 4), LARGE: EchoPool(LARGE, 4)}
    app = create_app(pools=pools)

    def work(i):
        client = app.test_client()
        sid = f"s{i}"
        for j in range(15):
            r = client.post("/chat", json={"message": f"msg {j} from {i}", "session_id": sid,
                                           "strategy": ["token", "heuristic", "hybrid", "perf"][(i + j) % 4]})
            assert r.status_code == 200, r.get_data(as_text=True)
        h = client.get(f"/history?session_id={sid}").get_json()
        assert len(h) == 10                       # trimmed to the last 10 messages (app.py:80-81)
        assert h[-2]["content"] == f"msg 14 from {i}"  # no cross-session interleaving

    run_threads(work)
