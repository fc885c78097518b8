"""Cross-rank pool protocol (pools.remote) on CPU (gloo): tagged requests with many in flight,
deadlines, dead-pool detection + failover, periodic health probes into the perf router, and the
token-id failover hand-off over the data plane.

Reference behaviour being matched: every device call is bounded (timeout=(5, 180)) and an error
fails over to the other device (/root/reference/src/models/nano.py:26-38, src/router.py:277-282);
liveness/readiness probing (src/models/server_manager.py:52-61,123-131)."""
import os
import socket
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.slow


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      DLLM_EMBEDDER="hash")
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _engine():
    from distributed_llm_amd.engine.llm_engine import LLMEngine
    return LLMEngine("tiny-llama-test", device="cpu", kv_cache_gb=0.05, max_num_seqs=16, seed=0)


def _groups():
    ctrl = dist.new_group([0, 1], backend="gloo")
    data = dist.new_group([0, 1], backend="gloo")
    return ctrl, data


def _worker(rank, world, port, scenario, q, env):
    os.environ.update(env)
    _init(rank, world, port)
    ctrl, data = _groups()
    try:
        if rank == 1:
            from distributed_llm_amd.pools.remote import PoolLeader
            PoolLeader(_engine(), ctrl, data, 0).serve()
            q.put({"rank": 1, "ok": True})
            return
        q.put(_ROUTER[scenario](ctrl, data))
    except Exception as e:  # noqa: BLE001 - surface in the parent
        import traceback
        q.put({"rank": rank, "error": f"{e!r}\n{traceback.format_exc()}"})
    finally:
        if scenario in ("concurrent", "handoff", "revive", "stuck_lock", "submit"):
            dist.destroy_process_group()
        else:
            q.close()
            q.join_thread()   # flush the result before skipping teardown
            os._exit(0)       # the peer is dead: do not wait in gloo teardown


def _router_concurrent(ctrl, data):
    """Long and short requests in flight at once: replies come back in completion order."""
    import threading
    from distributed_llm_amd.pools.remote import RemotePool
    rp = RemotePool("orin", 1, ctrl, data, max_new_tokens=4, timeout_s=120)
    done = []
    lock = threading.Lock()

    def call(tag, n):
        r = rp.process_batch([[{"role": "user", "content": f"request {tag}"}]], {"max_new_tokens": n})[0]
        with lock:
            done.append((tag, r))
    long_t = threading.Thread(target=call, args=("long", 200))
    long_t.start()
    time.sleep(0.3)   # the long request is decoding when the short ones arrive
    shorts = [threading.Thread(target=call, args=(f"s{i}", 3)) for i in range(3)]
    for t in shorts:
        t.start()
    for t in shorts + [long_t]:
        t.join(120)
    probe = rp.probe()
    rp.stop()
    return {"order": [t for t, _ in done], "errors": [r.get("error") for _, r in done],
            "tokens": {t: r.get("num_tokens") for t, r in done}, "probe": probe["ok"]}


def _router_kill(ctrl, data):
    """The pool process dies mid-request: the router fails over well inside the deadline, marks
    the pool dead, and its probes report the failure to the perf router."""
    from distributed_llm_amd.config import LARGE, SMALL
    from distributed_llm_amd.orchestrator import Router
    from distributed_llm_amd.pools.base import EnginePool
    from distributed_llm_amd.pools.remote import RemotePool
    health = []
    rp = RemotePool(LARGE, 1, ctrl, data, max_new_tokens=6, timeout_s=60)
    r = Router("heuristic", config={"cache_enabled": False}, pools={SMALL: EnginePool(SMALL, _engine(), 5),
                                                                   LARGE: rp})
    rp.on_health = lambda name, ok, rtt: (health.append(ok), r.on_pool_health(name, ok, rtt))
    rp.start_probes(interval_s=0.2, timeout_s=1.0, data_probe_every=0)
    time.sleep(0.6)
    t0 = time.perf_counter()
    payload, ntok, dev = r.route_query([{"role": "user", "content":
                                         "Write a Python function with recursion __die__ and explain it"}])
    dt = time.perf_counter() - t0
    time.sleep(1.0)
    return {"dev": dev, "ok": payload["ok"], "dt": dt, "alive": rp.alive, "health": health,
            "pool_health": r.pool_health.get(LARGE)}


def _router_hang(ctrl, data):
    """A request that never finishes: the caller gets an error payload at its deadline (the
    orchestrator then fails over), while health probes keep being answered."""
    from distributed_llm_amd.pools.remote import RemotePool
    rp = RemotePool("orin", 1, ctrl, data, max_new_tokens=4, timeout_s=2.0)
    t0 = time.perf_counter()
    rep = rp.process([{"role": "user", "content": "please __hang__ forever"}])
    dt = time.perf_counter() - t0
    probe = rp.probe(timeout=5.0)
    ok_after = rp.process([{"role": "user", "content": "and now a normal request"}])
    return {"err": rep.get("error", ""), "dt": dt, "probe": probe["ok"], "after": "response" in ok_after,
            "timeouts": rp.timeouts}


def _router_handoff(ctrl, data):
    """Failover hand-off as token ids over the data plane gives the same answer as text."""
    from distributed_llm_amd.engine.tokenizer import get_tokenizer
    from distributed_llm_amd.models.configs import get_model_config
    from distributed_llm_amd.pools.remote import RemotePool
    cfg = get_model_config("tiny-llama-test")
    rp = RemotePool("orin", 1, ctrl, data, max_new_tokens=7, timeout_s=60,
                    tokenizer=get_tokenizer(cfg.vocab, cfg.bos_id, cfg.eos_id))
    h = [{"role": "user", "content": "hand this prompt over as token ids"}]
    via_ids = rp.process_failover(h)
    via_text = rp.process(h)
    data_ping = rp.probe_data()
    rp.stop()
    return {"ids": via_ids.get("response"), "text": via_text.get("response"), "data_ping": data_ping["ok"]}


def _router_die_in_data_ping(ctrl, data):
    """The pool leader dies while a data-plane ping is in flight and a request is routed to it:
    the ping returns an error within its deadline (the data plane is retired, nothing blocks on
    its lock), the request fails over to the other tier well inside the request deadline."""
    import threading
    from distributed_llm_amd.config import LARGE, SMALL
    from distributed_llm_amd.orchestrator import Router
    from distributed_llm_amd.pools.base import EnginePool
    from distributed_llm_amd.pools.remote import RemotePool
    rp = RemotePool(LARGE, 1, ctrl, data, max_new_tokens=6, timeout_s=60, data_timeout_s=3.0)
    r = Router("heuristic", config={"cache_enabled": False}, pools={SMALL: EnginePool(SMALL, _engine(), 5),
                                                                   LARGE: rp})
    ping = {}

    def do_ping():
        t = time.perf_counter()
        ping["res"] = rp.probe_data(timeout=3.0)
        ping["dt"] = time.perf_counter() - t
    th = threading.Thread(target=do_ping)
    th.start()
    time.sleep(0.2)
    t0 = time.perf_counter()
    payload, ntok, dev = r.route_query([{"role": "user", "content":
                                         "Write a Python function with recursion and explain it step by step"}])
    dt = time.perf_counter() - t0
    th.join(30)
    # a later failover hand-off to this pool must not block on the data-plane lock either
    t1 = time.perf_counter()
    fo = rp.process_failover([{"role": "user", "content": "hello"}])
    return {"dev": dev, "ok": payload["ok"], "dt": dt, "ping_ok": ping["res"]["ok"], "ping_dt": ping["dt"],
            "fo_err": "error" in fo, "fo_dt": time.perf_counter() - t1, "alive": rp.alive}


def _router_revive(ctrl, data):
    """A pool whose receiver loop stalls (its first pings take 1.5 s against a 0.4 s probe
    deadline) is marked dead by the probes, but its transport is intact: after the stall the
    probes succeed again and the pool is put back in service."""
    from distributed_llm_amd.pools.remote import RemotePool
    health = []
    rp = RemotePool("orin", 1, ctrl, data, max_new_tokens=4, timeout_s=30, revive_after=2)
    rp.on_health = lambda name, ok, rtt: health.append(ok)
    rp.start_probes(interval_s=0.1, timeout_s=0.4, data_probe_every=0)
    t0 = time.perf_counter()
    dead_seen = False
    while time.perf_counter() - t0 < 20:
        if not rp.alive:
            dead_seen = True
        if dead_seen and rp.alive:
            break
        time.sleep(0.05)
    alive = rp.alive
    after = rp.process([{"role": "user", "content": "are you back?"}])
    rp._probe_stop.set()
    rp.stop()
    return {"dead_seen": dead_seen, "alive": alive, "revivals": rp.revivals, "after": "response" in after,
            "health": health}


def _router_stuck_data_lock(ctrl, data):
    """A data-plane transfer that never finishes holds the ordering lock: the failover hand-off
    gives up on the data plane after its deadline and ships the prompt as text instead."""
    from distributed_llm_amd.engine.tokenizer import get_tokenizer
    from distributed_llm_amd.models.configs import get_model_config
    from distributed_llm_amd.pools.remote import RemotePool
    cfg = get_model_config("tiny-llama-test")
    rp = RemotePool("orin", 1, ctrl, data, max_new_tokens=5, timeout_s=60, data_timeout_s=1.0,
                    tokenizer=get_tokenizer(cfg.vocab, cfg.bos_id, cfg.eos_id))
    rp._data_lock.acquire()             # as if a transfer were stuck forever
    # a health probe that finds the data plane busy skips (a long hand-off is not a failure)
    busy = rp.probe_data(timeout=0.3)
    busy_ok = busy.get("skipped") is not None and rp.data_error is None
    t0 = time.perf_counter()
    r = rp.process_failover([{"role": "user", "content": "hand me over"}])
    dt = time.perf_counter() - t0
    ping = rp.probe_data(timeout=1.0)
    rp.stop()
    return {"ok": "response" in r, "dt": dt, "retired": rp.data_error is not None, "ping_ok": ping["ok"],
            "busy_probe_skipped": busy_ok}


def _router_submit(ctrl, data):
    """Non-blocking submission (the event driver's path): one long and three short requests are
    submitted from ONE thread without waiting; each completes on its own (the shorts first) and
    reaches the completion queue exactly once; a failover hand-off is submitted the same way
    (token ids over the data plane)."""
    import queue
    from distributed_llm_amd.pools.remote import RemotePool
    from distributed_llm_amd.engine.tokenizer import get_tokenizer
    from distributed_llm_amd.models.configs import get_model_config
    cfg = get_model_config("tiny-llama-test")
    rp = RemotePool("orin", 1, ctrl, data, max_new_tokens=4, timeout_s=120,
                    tokenizer=get_tokenizer(cfg.vocab, cfg.bos_id, cfg.eos_id))
    q = queue.SimpleQueue()
    t0 = time.perf_counter()
    long_h = rp.submit_batch([[{"role": "user", "content": "request long"}]], {"max_new_tokens": 200}, notify=q.put)
    time.sleep(0.3)
    shorts = rp.submit_batch([[{"role": "user", "content": f"request s{i}"}] for i in range(3)],
                             {"max_new_tokens": 3}, notify=q.put)
    fo = rp.submit_failover([[{"role": "user", "content": "request fo"}]], notify=q.put)
    submit_s = time.perf_counter() - t0
    names = {id(long_h[0]): "long", id(fo[0]): "fo", **{id(h): f"s{i}" for i, h in enumerate(shorts)}}
    order = [names[id(q.get(timeout=120))] for _ in range(5)]
    extra = q.empty()
    res = rp.collect(long_h + shorts + fo)
    rp.stop()
    return {"order": order, "once": extra, "errors": [r.get("error") for r in res],
            "tokens": [r.get("num_tokens") for r in res], "submit_s": submit_s}


def _router_dead_sync(ctrl, data):
    """The leader dies on a request (fault injection).  Afterwards the router's control-plane use of
    that pool must fail fast instead of raising or blocking in gloo: ``sync()`` (the bench's
    window-opening barrier hand-off) fails the pool quietly, and a later submission completes at once
    with an error (the send checks the transport flag the receiver cleared)."""
    from distributed_llm_amd.pools.remote import RemotePool
    rp = RemotePool("orin", 1, ctrl, data, max_new_tokens=4, timeout_s=60)
    r = rp.process_batch([[{"role": "user", "content": "request __die__"}]])[0]
    t0 = time.perf_counter()
    while rp.transport_ok and time.perf_counter() - t0 < 20:
        time.sleep(0.05)
    sync_err = None
    try:
        rp.sync()
    except Exception as e:  # noqa: BLE001 - the regression: sync raised into the bench
        sync_err = repr(e)
    t1 = time.perf_counter()
    hs = rp.submit_batch([[{"role": "user", "content": "after"}]])
    res = rp.collect(hs)
    return {"first": r.get("error"), "transport_ok": rp.transport_ok, "sync_err": sync_err,
            "after_err": res[0].get("error"), "after_dt": time.perf_counter() - t1, "alive": rp.alive}


_ROUTER = {"dead_sync": _router_dead_sync, "concurrent": _router_concurrent, "kill": _router_kill, "hang": _router_hang,
           "handoff": _router_handoff, "data_die": _router_die_in_data_ping, "revive": _router_revive,
           "stuck_lock": _router_stuck_data_lock, "submit": _router_submit}


def _run(scenario, env=None, timeout=240):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, scenario, q, env or {})) for r in range(2)]
    for p in procs:
        p.start()
    outs = []
    try:
        for _ in range(2 if scenario in ("concurrent", "handoff", "revive", "stuck_lock", "submit") else 1):
            outs.append(q.get(timeout=timeout))
    finally:
        for p in procs:
            p.join(30)
            if p.is_alive():
                p.kill()
    for o in outs:
        assert "error" not in o or o.get("rank") is None, o.get("error")
    return [o for o in outs if o.get("rank") is None][0]


def test_concurrent_requests_complete_out_of_order():
    out = _run("concurrent")
    assert out["errors"] == [None] * 4
    assert out["order"][-1] == "long", out["order"]          # short requests overtook the long one
    assert out["tokens"]["long"] > out["tokens"]["s0"]
    assert out["probe"]


def test_dead_pool_fails_over_within_deadline():
    out = _run("kill", env={"DLLM_FAULT": "die_on=__die__"})
    assert out["ok"] and out["dev"] == "nano", out
    assert out["dt"] < 30.0, out                              # transport error, not the 60 s deadline
    assert out["alive"] is False
    assert False in out["health"] and out["pool_health"]["failures"] >= 1


def test_hung_request_times_out_and_pool_stays_usable():
    out = _run("hang", env={"DLLM_FAULT": "hang_on=__hang__,hang_s=4"})
    assert "timed out" in out["err"] and 1.5 < out["dt"] < 10.0, out
    assert out["probe"] and out["after"] and out["timeouts"] == 1


def test_failover_token_id_handoff_matches_text():
    out = _run("handoff")
    assert out["ids"] and out["ids"] == out["text"]
    assert out["data_ping"]


def test_leader_dies_during_data_ping_while_request_fails_over():
    out = _run("data_die", env={"DLLM_FAULT": "die_on_data_ping=1"})
    assert out["ok"] and out["dev"] == "nano", out
    assert out["dt"] < 30.0, out
    assert out["ping_ok"] is False and out["ping_dt"] < 8.0, out
    assert out["fo_err"] and out["fo_dt"] < 8.0 and out["alive"] is False, out


def test_pool_dead_by_probes_is_revived_when_probes_recover():
    out = _run("revive", env={"DLLM_FAULT": "ping_delay_n=3,ping_delay_s=1.5"})
    assert out["dead_seen"] and out["alive"] and out["revivals"] == 1, out
    assert out["after"], out
    assert False in out["health"] and out["health"][-1] is True


def test_stuck_data_plane_lock_falls_back_to_text():
    out = _run("stuck_lock")
    assert out["ok"] and out["dt"] < 20.0, out
    assert out["retired"] and out["ping_ok"] is False, out
    assert out["busy_probe_skipped"], out


def test_submit_batch_completes_each_request_on_its_own():
    out = _run("submit")
    assert out["errors"] == [None] * 5 and out["once"]
    assert out["order"][-1] == "long", out["order"]          # submitted earlier, finished last
    assert out["tokens"][0] == 200 and out["tokens"][1:4] == [3, 3, 3] and out["tokens"][4] == 4
    assert out["submit_s"] < 5.0                              # submission never waits for generation


def test_dead_leader_sync_and_sends_fail_fast():
    out = _run("dead_sync", env={"DLLM_FAULT": "die_on=__die__"})
    assert out["first"], out                                  # the request on the dying leader failed
    assert out["transport_ok"] is False and out["alive"] is False, out
    assert out["sync_err"] is None, out                       # sync() did not raise into the caller
    assert out["after_err"] and out["after_dt"] < 5.0, out    # a later send fails at once, no gloo wait
