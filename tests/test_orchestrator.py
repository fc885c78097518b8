"""Orchestrator contract (reference src/router.py) on echo pools: payload keys, response cache,
failover, context hashing, batch routing, fallback on routing exceptions."""
import hashlib

import pytest

from distributed_llm_amd.config import BENCHMARK_CFG, LARGE, PRODUCTION_CFG, SMALL
from distributed_llm_amd.orchestrator import Router, extract_text, history_to_query_and_context
from distributed_llm_amd.pools.base import EchoPool, FaultInjectingPool

MISS_KEYS = {"response", "raw", "cache_hit", "benchmark_mode", "routing_overhead_ms", "routing_method",
             "routing_confidence", "routing_reasoning", "ok"}
HIT_KEYS = {"response", "raw", "cache_hit", "routing_method", "routing_confidence", "routing_reasoning",
            "routing_overhead_ms", "ok"}


def pools():
    return {SMALL: EchoPool(SMALL, 8), LARGE: EchoPool(LARGE, 32)}


def test_history_split_and_hash():
    h = [{"role": "user", "content": " hi "}, {"role": "assistant", "content": "hello"},
         {"role": "user", "content": "  what is 2+2? "}]
    q, ctx, k = history_to_query_and_context(h, 6)
    assert q == "what is 2+2?"
    assert ctx == "user: hi\nassistant: hello"
    expect = hashlib.sha256("user:hi\nassistant:hello".encode()).hexdigest()[:16]
    assert k == expect
    assert history_to_query_and_context([], 6) == ("", None, "nohist")
    # no user message: whole history is context
    q, ctx, _ = history_to_query_and_context([{"role": "assistant", "content": "x"}], 6)
    assert q == "" and ctx == "assistant: x"


def test_extract_text_shapes():
    assert extract_text({"response": " a "}) == "a"
    assert extract_text({"message": {"content": "b"}}) == "b"
    assert extract_text({"error": "boom", "detail": "d"}) == "boom d"
    assert extract_text("  ") is None and extract_text(None) is None


def test_route_query_payload_keys_and_tokens():
    r = Router("heuristic", config=dict(BENCHMARK_CFG), benchmark_mode=True, pools=pools())
    payload, ntok, dev = r.route_query([{"role": "user", "content": "Thank you!"}])
    assert set(payload) == MISS_KEYS
    assert dev == SMALL and payload["routing_method"] == "heuristic" and payload["ok"] is True
    # reference: TokenCounter over the returned text (src/router.py:286) ...
    from distributed_llm_amd.router.tokens import TokenCounter
    assert ntok == TokenCounter().count_tokens({"role": "assistant", "content": payload["response"]})
    payload, ntok, dev = r.route_query([{"role": "user", "content": "Write a Python script that parses CSV"}])
    assert dev == LARGE and ntok == TokenCounter().count_tokens({"role": "assistant", "content": payload["response"]})
    # ... or the engine's generated-token count behind the tokens_from_engine flag
    r2 = Router("heuristic", config=dict(BENCHMARK_CFG, tokens_from_engine=True), benchmark_mode=True, pools=pools())
    assert r2.route_query([{"role": "user", "content": "Thank you!"}])[1] == 8


def test_response_cache_is_context_independent_like_reference():
    cfg = dict(PRODUCTION_CFG)
    r = Router("heuristic", config=cfg, pools=pools())
    a, _, _ = r.route_query([{"role": "user", "content": "hello"}])
    b, ntok, dev = r.route_query([{"role": "user", "content": "x"}, {"role": "assistant", "content": "y"},
                                  {"role": "user", "content": "  HELLO "}])
    assert a["cache_hit"] is False
    assert set(b) == HIT_KEYS and b["cache_hit"] is True and b["routing_method"] == "response_cache"
    assert b["response"] == a["response"] and dev == SMALL


def test_benchmark_mode_disables_response_cache():
    r = Router("token", config=dict(PRODUCTION_CFG), benchmark_mode=True, pools=pools())
    assert not r.enable_response_cache


def test_failover_to_other_tier():
    p = pools()
    p[SMALL] = FaultInjectingPool(p[SMALL], mode="error")
    r = Router("heuristic", config={"enable_failover": True, "cache_enabled": False}, pools=p)
    payload, ntok, dev = r.route_query([{"role": "user", "content": "Thank you!"}])
    assert dev == LARGE and payload["ok"] is True and payload["routing_method"] == "heuristic"


def test_failover_disabled_returns_error_payload():
    p = pools()
    p[SMALL] = FaultInjectingPool(p[SMALL], mode="error")
    r = Router("heuristic", config={"enable_failover": False, "cache_enabled": False}, pools=p)
    payload, ntok, dev = r.route_query([{"role": "user", "content": "Thank you!"}])
    assert dev == SMALL and payload["ok"] is False and "injected fault" in payload["response"]


def test_perf_feedback_reaches_perf_router():
    r = Router("perf", config={"cache_enabled": False}, pools=pools())
    for _ in range(3):
        r.route_query([{"role": "user", "content": "q"}])
    snap = r.query_router.router.snapshot()
    assert snap[SMALL]["n"] == 3


def test_routing_exception_falls_back_to_context_size():
    r = Router("token", config={"cache_enabled": False}, threshold_fallback=5, pools=pools())

    def boom(**kw):
        raise RuntimeError("router down")
    r.query_router.route_query = boom
    payload, _, dev = r.route_query([{"role": "user", "content": "a long enough message to exceed five tokens"}])
    assert payload["routing_method"] == "fallback_ctx_size" and payload["routing_confidence"] == 0.2
    assert dev == LARGE


def test_route_batch_matches_sequential_decisions():
    hs = [[{"role": "user", "content": q}] for q in ("Thank you!", "Write code for a web api", "hello there")]
    r1 = Router("heuristic", config={"cache_enabled": False}, pools=pools())
    r2 = Router("heuristic", config={"cache_enabled": False}, pools=pools())
    seq = [r1.route_query(h) for h in hs]
    bat = r2.route_batch(hs)
    assert [s[2] for s in seq] == [b[2] for b in bat]
    assert [s[0]["routing_method"] for s in seq] == [b[0]["routing_method"] for b in bat]


def test_route_batch_failover():
    p = pools()
    p[LARGE] = FaultInjectingPool(p[LARGE], mode="error")
    r = Router("heuristic", config={"cache_enabled": False}, pools=p)
    out = r.route_batch([[{"role": "user", "content": "Write a Python function"}]])
    assert out[0][2] == SMALL and out[0][0]["ok"]


def test_penalise_failed_primary_option():
    p = pools()
    p[SMALL] = FaultInjectingPool(p[SMALL], mode="error")
    r = Router("perf", config={"cache_enabled": False, "penalise_failed_primary": True}, pools=p)
    r.route_query([{"role": "user", "content": "q"}])
    snap = r.query_router.router.snapshot()
    assert snap[SMALL]["n"] == 1 and snap[LARGE]["n"] == 1


class _DyingPool(EchoPool):
    """A remote-pool stand-in: answers until ``die()``, then errors and reports ``alive`` False
    (as pools.remote.RemotePool does once its process is gone)."""

    def __init__(self, name):
        super().__init__(name, 20)
        self.alive = True
        self.calls = 0

    def die(self):
        self.alive = False

    def process(self, history):
        self.calls += 1
        if not self.alive:
            return {"error": "pool process died"}
        return super().process(history)


def test_perf_router_with_exploration_stops_choosing_a_dead_pool():
    """BASELINE config 4's perf-router failover: with ``perf_explore`` the large tier is tried,
    its death fails turns over to the small tier (none lost), failures are charged to it
    (``penalise_failed_primary``) and the perf router stops choosing it; a pool reported down
    is skipped up front (no failed attempt per turn)."""
    large = _DyingPool(LARGE)
    r = Router("perf", config={"cache_enabled": False, "perf_explore": True, "penalise_failed_primary": True},
               pools={SMALL: EchoPool(SMALL, 6), LARGE: large})
    h = [{"role": "user", "content": "hello"}]
    devs = [r.route_query(h)[2] for _ in range(2)]
    assert devs == [SMALL, LARGE]            # no stats -> small; then the unseen large is explored
    large.die()
    out = [r.route_query(h) for _ in range(6)]
    assert all(p["ok"] and d == SMALL for p, _, d in out)   # zero lost turns
    calls = large.calls
    decisions = [r.query_router.route_query("hello").device for _ in range(3)]
    assert decisions == [SMALL] * 3          # the failure penalty keeps the perf router away
    r.route_batch([h, h])
    assert large.calls == calls              # a pool that is down is not even attempted


def test_dead_pool_skipped_up_front_for_any_strategy():
    large = _DyingPool(LARGE)
    r = Router("heuristic", config={"cache_enabled": False}, pools={SMALL: EchoPool(SMALL), LARGE: large})
    q = [{"role": "user", "content": "Write a Python function for knapsack with dynamic programming"}]
    assert r.route_query(q)[2] == LARGE
    large.die()
    calls = large.calls
    p, _, d = r.route_query(q)
    assert d == SMALL and p["ok"] and p["failover_from"] == LARGE and large.calls == calls
    res = r.route_batch([q, q])
    assert all(x[2] == SMALL and x[0]["failover_from"] == LARGE for x in res) and large.calls == calls
