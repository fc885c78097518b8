"""bench.py driver contract on CPU (gloo): one JSON line from rank 0 with the required keys, for
the default replicated topology (dp) and the disjoint-pool topology (small replicas + large TP)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


# every N defaults to config-2 replicas (a weak-scaling curve of one workload); BASELINE's
# multi-GPU configs by flag (3 at 2 ranks, 4 at 4-8); config 5 = the large TP group over every
# rank with a small replica co-located on each
@pytest.mark.parametrize("n,extra,par,cfg", [(1, [], "dp1", 2), (2, [], "dp2", 2),
                                             (2, ["--baseline-config", "3"], "pools:small1xtp1+large1xtp1", 3),
                                             (4, ["--topology", "pools"], "pools:small2xtp1+large1xtp2", 4),
                                             (2, ["--baseline-config", "5"], "colocated:small2xtp1+large1xtp2", 5),
                                             (1, ["--topology", "tiers"], "dp1-colocated", 2)])
def test_bench_json_line(n, extra, par, cfg):
    args = ["bench.py", "--cpu", "--gpus", str(n), "--steps", "1", "--warmup", "1", "--convs", "2",
            "--small-new", "4", "--large-new", "6"] + extra
    if n > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
               "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
    else:
        cmd = [sys.executable] + args
    env = dict(os.environ, DLLM_EMBEDDER="hash", OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert KEYS <= set(out)
    assert out["n_gpus"] == n and out["steps"] == 1 and out["warmup"] == 1
    assert out["value"] > 0 and out["higher_is_better"] is True
    assert out["scaling"] == ("weak" if cfg == 2 else "config")
    assert out["per_gpu_tok_s"] * n == pytest.approx(out["value"], rel=1e-3)
    assert 0 < out["init_s"] <= out["startup_s"]
    assert out["config"]["parallelism"].startswith(par)
    if out["config"]["turn_pipelining"]:
        # pipelined (the 1-GPU default): the window counts the turns completed inside it
        assert out["requests"] >= 2 * n - 2 and out["config"]["turn_pipelining"] == "event-driver"
    else:
        assert out["requests"] == 2 * n
    assert out["p50_latency_ms"] > 0
    assert out["baseline_config"] == cfg
    cc = out["collective_cross_check"]
    if n > 1 and cfg == 2:   # replicas also reduce through the process group (gloo here, RCCL on a node)
        assert cc["backend"] == "gloo" and cc["ranks"] == n and cc["matches_store"] is True
    else:
        assert cc is None
    lay = out["layout"]
    assert set(lay) >= {"small", "large"} and lay["small"]["replicas"] and lay["large"]["replicas"]
    if cfg == 5:   # every rank hosts a small replica AND a shard of the large TP group
        assert lay["colocated"] and lay["large"]["replicas"] == [list(range(n))]
        assert lay["small"]["replicas"] == [[r] for r in range(n)]
    assert out["per_stream_vs_baseline"] is None or out["per_stream_vs_baseline"] > 0


def test_bench_survives_pool_leader_death():
    """Pools topology on 4 CPU ranks (small replicas [0], [1]; large TP=2 on [2, 3]) with the large
    leader killed by fault injection after its first request batch: plain processes (not torchrun,
    whose agent would tear every rank down), the survivors exit 0, no turn is lost (failover to the
    small replicas), and rank 0 reduces the survivors' results through the rendezvous store."""
    world, port = 4, _port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), DLLM_EMBEDDER="hash", OMP_NUM_THREADS="1", DLLM_FAULT="die_rank=2,die_after=1")
        procs.append(subprocess.Popen([sys.executable, "bench.py", "--cpu", "--gpus", str(world), "--steps", "3",
                                       "--warmup", "1", "--convs", "3", "--small-new", "4", "--large-new", "6",
                                       "--strategy", "hybrid", "--topology", "pools"], cwd=ROOT, env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.DEVNULL, text=True))
    outs = [p.communicate(timeout=300)[0] for p in procs]
    assert [p.returncode for p in procs] == [0, 0, 17, 0]
    line = [ln for ln in outs[0].splitlines() if ln.startswith("{")]
    out = json.loads(line[0])
    ev = out["pool_events"]
    assert ev["dead_ranks"] == [2] and ev["failed_tiers"] == ["orin"] and ev["degraded"]
    # pipelined (the default): the window closes once steps x convs turns have completed in it
    assert ev["failovers"] > 0 and ev["lost_turns"] == 0 and out["requests"] >= 3 * world * 3


def test_bench_event_driven_turn_pipelining():
    """``--pipeline 2``: one driver thread keeps every conversation's next turn in flight through the
    engine's non-blocking submission; the timed window counts completed turns (about steps x convs)."""
    args = [sys.executable, "bench.py", "--cpu", "--steps", "2", "--warmup", "1", "--convs", "4",
            "--small-new", "4", "--large-new", "6", "--pipeline", "2", "--admit-every", "4"]
    env = dict(os.environ, DLLM_EMBEDDER="hash", OMP_NUM_THREADS="1")
    r = subprocess.run(args, cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert out["config"]["turn_pipelining"] == "event-driver" and out["config"]["admit_every"] == 4
    assert out["value"] > 0 and out["requests"] >= 2 * 4 - 4 and out["pool_events"]["lost_turns"] == 0


def test_bench_helpers_busy_sampler_and_kv_placement():
    """The busy sampler degrades to None where amdsmi / a GPU is missing (this container), and the
    KV placement shares are deltas of the block manager's counters over the window."""
    from distributed_llm_amd.bench.power import BusySampler
    b = BusySampler(0, hz=100.0).start()
    assert b.stop() is None or 0.0 <= b.stop() <= 100.0
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    st0 = [{"contiguous_allocs": 10, "segment_allocs": 1, "fresh_allocs": 20, "run_miss_held": 2}]
    st1 = [{"contiguous_allocs": 70, "segment_allocs": 3, "fresh_allocs": 100, "run_miss_held": 10,
            "inplace_evictions": 20}]
    got = bench.kv_placement(st0, st1)
    assert {k: got[k] for k in ("new_blocks", "run_share", "segment_share")} == \
        {"new_blocks": 80, "run_share": 0.75, "segment_share": 0.025}
    assert got["run_miss_held_share"] == 0.1 and got["inplace_share"] == 0.25 and got["run_miss_hot_share"] == 0.0
    assert bench.kv_placement([{}], [{}])["run_share"] is None


def test_peak_mem_helper_gpu_branch(monkeypatch):
    """The GPU branch of the per-rank memory report runs without a GPU here (allocator stubbed):
    the helper must not depend on module-level imports that bench.py defers to main()."""
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    monkeypatch.setattr(torch.cuda, "max_memory_allocated", lambda *a, **k: 3 * 2**30)
    assert bench._peak_mem_gb(True) == 3.0
    assert bench._peak_mem_gb(False) is None
