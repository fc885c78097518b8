"""Multi-pool node topology on CPU (gloo, world 3): router + small pool on rank 0, large pool as a
TP=2 group on ranks 1-2 reached over point-to-point messages.  Routed results must equal a
single-process run with local engines; probes return stats; a stopped pool fails over."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HISTS = [[{"role": "user", "content": "Thank you!"}],
         [{"role": "user", "content": "Write a Python function for knapsack with dynamic programming"}],
         [{"role": "user", "content": "hello there"}],
         [{"role": "user", "content": "Compare BFS and DFS in depth"}]]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _specs():
    from distributed_llm_amd.config import LARGE, SMALL
    from distributed_llm_amd.parallel.cluster import TierSpec
    return {SMALL: TierSpec("tiny-llama-test", 5, kv_cache_gb=0.05, max_num_seqs=8),
            LARGE: TierSpec("tiny-moe-test", 7, kv_cache_gb=0.05, max_num_seqs=8)}


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      DLLM_EMBEDDER="hash")
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from distributed_llm_amd.config import LARGE, SMALL
        from distributed_llm_amd.orchestrator import Router
        from distributed_llm_amd.parallel.cluster import Cluster, Topology
        topo = Topology({SMALL: [[0]], LARGE: [[1, 2]]})
        cl = Cluster(topo, _specs(), device="cpu")
        if rank == 0:
            pools = cl.router_pools()
            r = Router("heuristic", config={"cache_enabled": False}, pools=pools)
            cl.sync()
            res = r.route_batch(HISTS)
            probe = pools[LARGE].probe()
            cl.sync()
            pools[LARGE].stop()  # pool goes away -> failover to the small tier
            after = r.route_query(HISTS[1])
            q.put({"res": [(p["response"], n, d) for p, n, d in res], "probe": probe,
                   "after": (after[2], after[0]["ok"]), "syncs": len(cl.sync_times)})
        else:
            cl.serve()
            q.put({"rank": rank, "syncs": len(cl.sync_times)})
    finally:
        dist.destroy_process_group()


def test_cluster_routes_across_ranks_and_fails_over():
    os.environ["DLLM_EMBEDDER"] = "hash"
    from distributed_llm_amd.config import LARGE, SMALL
    from distributed_llm_amd.engine.llm_engine import LLMEngine
    from distributed_llm_amd.orchestrator import Router
    from distributed_llm_amd.pools.base import EnginePool
    sp = _specs()
    local = {t: EnginePool(t, LLMEngine(s.model, device="cpu", kv_cache_gb=0.05, max_num_seqs=8), s.max_new_tokens)
             for t, s in sp.items()}
    ref = [(p["response"], n, d) for p, n, d in
           Router("heuristic", config={"cache_enabled": False}, pools=local).route_batch(HISTS)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    main = [o for o in outs if "res" in o][0]
    assert [tuple(x) for x in main["res"]] == ref
    assert {d for _, _, d in ref} == {SMALL, LARGE}
    assert main["probe"]["ok"] and main["probe"]["model"] == "tiny-moe-test"
    assert tuple(main["after"]) == (SMALL, True)
    assert all(o["syncs"] == 2 for o in outs)


def test_default_topologies():
    from distributed_llm_amd.config import LARGE, SMALL
    from distributed_llm_amd.parallel.cluster import default_topology
    assert default_topology(1).replicas == {SMALL: [[0]], LARGE: [[0]]}
    assert default_topology(2).replicas == {SMALL: [[0]], LARGE: [[1]]}
    assert default_topology(8).replicas == {SMALL: [[0], [1], [2], [3]], LARGE: [[4, 5, 6, 7]]}
    assert default_topology(8, large_tp=2).replicas[LARGE] == [[4, 5], [6, 7]]


def _coloc_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      DLLM_EMBEDDER="hash")
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from distributed_llm_amd.config import LARGE, SMALL
        from distributed_llm_amd.orchestrator import Router
        from distributed_llm_amd.parallel.cluster import Cluster, default_topology
        topo = default_topology(world, colocated=True)
        cl = Cluster(topo, _specs(), device="cpu")
        assert len(cl.engines) == 2      # a small replica and a large TP shard on every rank
        if rank == 0:
            pools = cl.router_pools()
            r = Router("heuristic", config={"cache_enabled": False}, pools=pools)
            cl.sync()
            res = r.route_batch(HISTS * 2)
            cl.sync()
            cl.shutdown()
            q.put({"res": [(p["response"], n, d) for p, n, d in res], "syncs": len(cl.sync_times)})
        else:
            cl.serve()
            q.put({"rank": rank, "syncs": len(cl.sync_times)})
    finally:
        dist.destroy_process_group()


def test_colocated_pools_share_ranks():
    """BASELINE config 5's layout on CPU: the large pool is one TP group over ranks 0-1 and each
    rank also hosts a small replica (two engines, two serving loops per pool rank).  Both tiers
    serve, every rank joins each node sync exactly once and exits cleanly."""
    from distributed_llm_amd.config import LARGE, SMALL
    from distributed_llm_amd.parallel.cluster import default_topology
    assert default_topology(8, colocated=True).replicas == {SMALL: [[r] for r in range(8)],
                                                            LARGE: [list(range(8))]}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_coloc_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    main = [o for o in outs if "res" in o][0]
    assert {d for _, _, d in main["res"]} == {SMALL, LARGE}
    assert all(n > 0 for _, n, _ in main["res"])
    assert all(o["syncs"] == 2 for o in outs)
