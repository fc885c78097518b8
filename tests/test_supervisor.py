"""Failure detection and recovery on real worker processes (echo pools, CPU):
supervisor bring-up / health, crash detection + restart, lazy restart from the pool client,
watchdog restart, and orchestrator failover when a pool process is killed."""
import os
import signal
import socket
import time

import pytest

from distributed_llm_amd.config import LARGE, SMALL
from distributed_llm_amd.pools.base import HTTPPool
from distributed_llm_amd.pools.supervisor import PoolSpec, Supervisor


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture()
def sup(tmp_path):
    s = Supervisor([PoolSpec(SMALL, _port(), kind="echo", max_new_tokens=8),
                    PoolSpec(LARGE, _port(), kind="echo", max_new_tokens=16)],
                   log_dir=str(tmp_path / "logs"), startup_timeout_s=120)
    yield s
    s.stop_all()


def _crash(sup, name):
    p = sup.procs[name]
    os.killpg(p.pid, signal.SIGKILL)  # the process group the supervisor created for this worker
    p.wait(timeout=30)
    assert not sup.alive(name)


HIST = [{"role": "user", "content": "hello there"}]


def test_start_health_crash_restart(sup):
    assert sup.start_all() == {SMALL: True, LARGE: True}
    assert sup.is_running(SMALL) and sup.is_running(LARGE)
    pool = HTTPPool(SMALL, sup.specs[SMALL].url)
    assert "response" in pool.process(HIST)
    _crash(sup, SMALL)
    assert "error" in pool.process(HIST)           # detection: the client sees an error dict
    assert sup.ensure(SMALL) and sup.restarts[SMALL] == 1
    assert "response" in pool.process(HIST)


def test_lazy_restart_from_client(sup):
    sup.start_all()
    pool = HTTPPool(SMALL, sup.specs[SMALL].url, supervisor=sup)
    _crash(sup, SMALL)
    # reference nano.py:19-21: the client restarts a server whose port is closed before posting
    assert "response" in pool.process(HIST)


def test_watchdog_restarts_dead_worker(sup):
    sup.start_all()
    sup.watch(interval_s=0.2)
    _crash(sup, LARGE)
    t0 = time.time()
    while time.time() - t0 < 60 and not sup.is_running(LARGE):
        time.sleep(0.2)
    assert sup.is_running(LARGE) and sup.restarts[LARGE] >= 1


def test_router_fails_over_when_pool_process_dies(sup):
    from distributed_llm_amd.config import BENCHMARK_CFG
    from distributed_llm_amd.orchestrator import Router
    sup.start_all()
    pools = {SMALL: HTTPPool(SMALL, sup.specs[SMALL].url), LARGE: HTTPPool(LARGE, sup.specs[LARGE].url)}
    r = Router(strategy="token", config=dict(BENCHMARK_CFG, enable_failover=True), pools=pools)
    _, _, dev = r.route_query(HIST)
    assert dev == SMALL                               # short query -> small tier
    _crash(sup, SMALL)
    payload, tokens, dev = r.route_query(HIST)
    assert dev == LARGE and payload.get("ok") and tokens > 0   # failover served it


def test_tensor_parallel_pool_worker_matches_tp1(tmp_path):
    """A tp=2 pool: the supervisor launches torchrun (2 ranks, gloo on CPU); rank 0 serves HTTP and
    leads the scheduler, rank 1 follows it in lockstep.  /query must give the same greedy tokens
    as the in-process TP=1 engine (reference ServerManager.start_server brings up ONE working
    server: /root/reference/src/models/server_manager.py:66-142)."""
    from distributed_llm_amd.engine.llm_engine import LLMEngine
    from distributed_llm_amd.pools.base import EnginePool
    args = ["--device", "cpu", "--kv-gb", "0.05", "--max-num-seqs", "8"]
    s = Supervisor([PoolSpec(LARGE, _port(), kind="engine", model="tiny-llama-test", max_new_tokens=9, tp=2,
                             extra_args=args)], log_dir=str(tmp_path / "logs"), startup_timeout_s=240)
    try:
        assert s.start(LARGE), open(tmp_path / "logs" / f"{LARGE}.log").read()[-3000:]
        pool = HTTPPool(LARGE, s.specs[LARGE].url, timeout_s=120)
        hist = [{"role": "user", "content": "tensor parallel pools answer like one GPU"}]
        got = pool.process(hist)
        # concurrent requests join the TP pool's continuous batch (mirrored scheduler)
        import concurrent.futures as cf
        with cf.ThreadPoolExecutor(4) as ex:
            many = list(ex.map(pool.process, [[{"role": "user", "content": f"question {i}"}] for i in range(4)]))
    finally:
        s.stop_all()
    ref = EnginePool(LARGE, LLMEngine("tiny-llama-test", device="cpu", kv_cache_gb=0.05, max_num_seqs=8),
                     max_new_tokens=9).process(hist)
    assert "response" in got, got
    assert got["response"] == ref["response"]
    assert all("response" in m for m in many), many


def test_supervised_pool_spec_restarts_dead_worker(tmp_path):
    """Topology kind "supervised" (pools/factory.py): the router owns the worker processes and the
    next request to a pool whose process died restarts it (reference src/models/nano.py:19-21)."""
    from distributed_llm_amd.pools.factory import build_pools
    spec = {SMALL: {"kind": "supervised", "port": _port(), "worker_kind": "echo", "max_new_tokens": 8,
                    "log_dir": str(tmp_path / "logs"), "startup_timeout_s": 120},
            LARGE: {"kind": "supervised", "port": _port(), "worker_kind": "echo", "max_new_tokens": 16,
                    "log_dir": str(tmp_path / "logs"), "startup_timeout_s": 120}}
    pools = build_pools(spec)
    sup = pools[SMALL].server_manager.supervisor
    try:
        assert sup is pools[LARGE].server_manager.supervisor
        assert pools[LARGE].process(HIST)["response"]
        _crash(sup, LARGE)
        r = pools[LARGE].process(HIST)          # lazy restart before the call
        assert r["response"] and sup.restarts[LARGE] == 1 and sup.alive(LARGE)
    finally:
        sup.stop_all()


def test_supervised_topology_file_parses_without_starting():
    """The shipped config-4 supervised topology builds two supervised pools (TP=4 large tier)."""
    import json
    import os
    from distributed_llm_amd.pools.factory import build_pools
    path = os.path.join(os.path.dirname(__file__), "..", "distributed_llm_amd", "data", "topologies",
                        "supervised_pools_8gpu.json")
    spec = {k: dict(v, start=False) for k, v in json.load(open(path)).items() if not k.startswith("_")}
    pools = build_pools(spec)
    sup = pools[SMALL].server_manager.supervisor
    try:
        assert set(pools) == {SMALL, LARGE}
        assert sup.specs[LARGE].tp == 4 and sup.specs[LARGE].gpus == [4, 5, 6, 7]
        assert not sup.alive(SMALL) and not sup.alive(LARGE)
    finally:
        sup.stop_all()
