"""Event-driven dispatch (``Router.dispatch_batch`` / ``finish_ticket``) with non-blocking failover.

Reference behaviour: a device error fails the request over to the other device on the request's
own thread (src/router.py:277-282), so one failed turn never holds up another conversation.  Here
one driver thread serves every conversation; the failover generation must therefore be
re-submitted (a ticket back in flight), not run inline on the driver.
"""
import queue
import threading
import time

from distributed_llm_amd.config import BENCHMARK_CFG, LARGE, SMALL
from distributed_llm_amd.orchestrator import Router
from distributed_llm_amd.pools.base import EchoPool, FaultInjectingPool, PoolHandle, ThreadSubmit
from distributed_llm_amd.pools.remote import ReplicatedPool


class SlowEcho(EchoPool):
    """Echo that takes ``delay_s`` for prompts containing ``marker`` (e.g. a failover target)."""

    def __init__(self, name, marker="", delay_s=1.0, **kw):
        super().__init__(name, **kw)
        self.marker, self.slow = marker, delay_s

    def process(self, history):
        from distributed_llm_amd.pools.base import format_prompt
        if self.marker and self.marker in format_prompt(history):
            time.sleep(self.slow)
        return super().process(history)


def _conv(text):
    return [{"role": "user", "content": text}]


def test_failover_is_resubmitted_not_run_on_the_driver():
    """The large tier errors; finishing the failed ticket re-submits it to the small tier and
    returns at once (the failover takes 1 s); the re-submitted ticket then completes with
    ``failover_from`` = large, served by small, and its client latency covers both attempts."""
    pools = {SMALL: SlowEcho(SMALL, marker="knapsack", delay_s=1.0),
             LARGE: FaultInjectingPool(EchoPool(LARGE), mode="error")}
    r = Router("heuristic", config=dict(BENCHMARK_CFG), pools=pools)
    q = queue.SimpleQueue()
    t = r.dispatch_batch([_conv("Write a Python function for knapsack with dynamic programming")], notify=q.put)[0]
    assert t["device"] == LARGE
    h = q.get(timeout=10)
    assert h is t["handle"]
    t0 = time.perf_counter()
    assert r.finish_ticket(t, notify=q.put) is None          # back in flight on the small tier
    assert time.perf_counter() - t0 < 0.5
    assert t["device"] == SMALL and t["failover_from"] == LARGE
    h2 = q.get(timeout=10)
    assert h2 is t["handle"] and h2 is not h
    payload, ntok, dev = r.finish_ticket(t, notify=q.put)
    assert dev == SMALL and payload["failover_from"] == LARGE and payload["ok"] and ntok > 0
    assert t["latency_ms"] >= 1000.0


def test_one_failing_turn_does_not_block_other_conversations():
    """Two conversations: A's large-tier turn fails and its failover takes 1.5 s; B (small tier,
    fast) keeps completing turns meanwhile.  Driven by one thread, as bench.py's event driver."""
    pools = {SMALL: SlowEcho(SMALL, marker="knapsack", delay_s=1.5),
             LARGE: FaultInjectingPool(EchoPool(LARGE), mode="error")}
    r = Router("heuristic", config=dict(BENCHMARK_CFG), pools=pools)
    q = queue.SimpleQueue()
    hist = {"A": _conv("Write a Python function for knapsack with dynamic programming"), "B": _conv("Thank you!")}
    inflight, done_at = {}, {"A": [], "B": []}
    for name, t in zip(hist, r.dispatch_batch(list(hist.values()), notify=q.put)):
        inflight[id(t["handle"])] = (name, t)
    t_start = time.perf_counter()
    while time.perf_counter() - t_start < 10 and not done_at["A"]:
        try:
            h = q.get(timeout=0.05)
        except queue.Empty:
            continue
        name, t = inflight.pop(id(h))
        res = r.finish_ticket(t, notify=q.put)
        if res is None:
            inflight[id(t["handle"])] = (name, t)
            continue
        done_at[name].append(time.perf_counter() - t_start)
        hist[name] = hist[name] + [{"role": "assistant", "content": res[0]["response"]},
                                   {"role": "user", "content": "Thank you!" if name == "B" else "knapsack again"}]
        if name == "B":
            nt = r.dispatch_batch([hist[name]], notify=q.put)[0]
            inflight[id(nt["handle"])] = (name, nt)
    assert done_at["A"] and done_at["A"][0] >= 1.4
    # B finished several turns while A's failover was running
    assert sum(1 for x in done_at["B"] if x < done_at["A"][0]) >= 3, done_at


def test_dispatch_sends_a_dead_tier_to_the_other_tier_up_front():
    class Dead(EchoPool):
        alive = False
    pools = {SMALL: EchoPool(SMALL), LARGE: Dead(LARGE)}
    r = Router("heuristic", config=dict(BENCHMARK_CFG), pools=pools)
    q = queue.SimpleQueue()
    t = r.dispatch_batch([_conv("Write a Python function for knapsack with dynamic programming")], notify=q.put)[0]
    assert t["device"] == SMALL and t["failover_from"] == LARGE
    q.get(timeout=10)
    payload, _, dev = r.finish_ticket(t, notify=q.put)
    assert dev == SMALL and payload["failover_from"] == LARGE and pools[LARGE].calls == 0


def test_replicated_pool_submit_balances_and_collects():
    reps = [EchoPool(SMALL, tokens_per_reply=4), EchoPool(SMALL, tokens_per_reply=4)]
    rp = ReplicatedPool(SMALL, reps)
    q = queue.SimpleQueue()
    hs = rp.submit_batch([_conv(f"hello {i}") for i in range(6)], notify=q.put)
    got = {id(q.get(timeout=10)) for _ in hs}
    assert got == {id(h) for h in hs} and q.empty()
    res = rp.collect(hs)
    assert all(x["response"].endswith(str(i)) or str(i) in x["response"] for i, x in enumerate(res))
    assert reps[0].calls == 3 and reps[1].calls == 3 and rp.inflight == [0, 0]


def test_pool_handle_notifies_exactly_once():
    calls = []
    h = PoolHandle(calls.append)
    assert h.complete({"response": "a"}) and not h.complete({"error": "late"})
    assert calls == [h] and h.payload() == {"response": "a"}


def test_thread_submit_reports_a_raising_pool_as_errors():
    class Boom(EchoPool):
        def process_batch(self, histories):
            raise RuntimeError("boom")
    hs = Boom(SMALL).submit_batch([_conv("x"), _conv("y")])
    for h in hs:
        assert h.done.wait(10)
    assert all("boom" in h.payload()["error"] for h in hs)
    assert isinstance(Boom(SMALL), ThreadSubmit) and threading.active_count() >= 1


def test_replicated_pool_load_returns_to_zero_without_collect():
    """handles that are never collected must not leak bookkeeping or skew the load."""
    reps = [EchoPool(SMALL, tokens_per_reply=2), EchoPool(SMALL, tokens_per_reply=2)]
    rp = ReplicatedPool(SMALL, reps)
    for rnd in range(20):
        q = queue.SimpleQueue()
        hs = rp.submit_batch([_conv(f"r{rnd} q{i}") for i in range(8)], notify=q.put)
        for _ in hs:
            q.get(timeout=10)
        del hs
    assert rp.inflight == [0, 0]
    assert not any(k.startswith("_owner") or k.startswith("_released") for k in vars(rp))


def test_replicated_pool_collect_before_done_counts_once():
    reps = [SlowEcho(SMALL, marker="slow", delay_s=0.5), SlowEcho(SMALL, marker="slow", delay_s=0.5)]
    rp = ReplicatedPool(SMALL, reps)
    q = queue.SimpleQueue()
    hs = rp.submit_batch([_conv("slow a"), _conv("slow b")], notify=q.put)
    rp.collect(hs)             # not done yet: released now ...
    assert rp.inflight == [0, 0]
    for _ in hs:               # ... and the later completion callbacks do not count again
        q.get(timeout=10)
    assert rp.inflight == [0, 0]


def test_both_tiers_down_reports_like_route_query():
    """an up-front failover whose target fails too reports the primary's error and no
    failover, as the blocking route_query does."""
    class Dead(FaultInjectingPool):
        alive = False
    pools = {SMALL: FaultInjectingPool(EchoPool(SMALL), mode="error"), LARGE: Dead(EchoPool(LARGE), mode="error")}
    r = Router("heuristic", config=dict(BENCHMARK_CFG), pools=pools)
    q = queue.SimpleQueue()
    t = r.dispatch_batch([_conv("Write a Python function for knapsack with dynamic programming")], notify=q.put)[0]
    assert t["device"] == SMALL and t["failover_from"] == LARGE
    if t.get("handle") is not None:
        q.get(timeout=10)
    payload, _, dev = r.finish_ticket(t, notify=q.put)
    assert dev == LARGE and "failover_from" not in payload and not payload["ok"]
    assert "unavailable" in str(payload.get("response", "")) + str(payload.get("raw", ""))
