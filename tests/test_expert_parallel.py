"""Expert parallelism on CPU (gloo): the all-to-all MoE layer equals the single-rank MoE FFN on the
same tokens (2 and 4 ranks, uneven token counts, a rank with no tokens), and an EP=2 Mixtral-style
engine generates the TP=1 engine's greedy tokens."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from distributed_llm_amd.parallel.expert_parallel import token_slice


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _layer_case(T, E=8, H=32, I=48, k=2, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = (torch.randn(T, H, generator=g) * 0.5).to(torch.bfloat16)
    logits = torch.randn(T, E, generator=g)
    w13 = (torch.randn(E, 2 * I, H, generator=g) * 0.1).to(torch.bfloat16)
    w2 = (torch.randn(E, H, I, generator=g) * 0.1).to(torch.bfloat16)
    return x, logits, w13, w2, k


def _layer_worker(rank, world, port, T, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from distributed_llm_amd import ops
        from distributed_llm_amd.parallel.expert_parallel import all_gather_rows, ep_moe_ffn
        x, logits, w13, w2, k = _layer_case(T)
        E = w13.shape[0]
        lo, hi = token_slice(T, rank, world)
        ids, w = ops.moe_gate(logits[lo:hi], k)
        es = slice(rank * E // world, (rank + 1) * E // world)
        yl = ep_moe_ffn(x[lo:hi], ids, w, w13[es], w2[es], E, None, world)
        y = all_gather_rows(yl, T, None, world)
        # by value: a shared-memory tensor dies with this process if the parent reads it late
        q.put((rank, y.float().numpy().copy()))
    finally:
        dist.destroy_process_group()


def _spawn(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, *args, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_token_slice_partitions():
    for T in (0, 1, 5, 16, 17):
        for P in (1, 2, 3, 4, 8):
            parts = [token_slice(T, r, P) for r in range(P)]
            assert parts[0][0] == 0 and parts[-1][1] == T
            assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
            assert max(h - l for l, h in parts) - min(h - l for l, h in parts) <= 1


@pytest.mark.parametrize("world,T", [(2, 13), (4, 3)])   # T=3 on 4 ranks: one rank has no tokens
def test_ep_layer_matches_single_rank(world, T):
    from distributed_llm_amd import ops
    x, logits, w13, w2, k = _layer_case(T)
    ids, w = ops.moe_gate(logits, k)
    want = ops.moe_ffn(x, ids, w, w13, w2).float()
    res = _spawn(_layer_worker, world, T)
    res = {r: torch.from_numpy(v) for r, v in res.items()}
    for r in range(world):
        torch.testing.assert_close(res[r], want, atol=2e-2, rtol=2e-2)
    assert all(torch.equal(res[0], res[r]) for r in range(world))


PROMPTS = ["user: hello there", "user: explain expert parallelism step by step", "y" * 50]


def _engine_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      DLLM_MOE_PARALLEL="ep", DLLM_EP_MIN_TOKENS="1")
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from distributed_llm_amd.engine.llm_engine import LLMEngine
        from distributed_llm_amd.engine.sampling import SamplingParams
        from distributed_llm_amd.parallel.comm import make_tp_groups
        eng = LLMEngine("tiny-moe-test", device="cpu", par=make_tp_groups(world), kv_cache_gb=0.05, max_num_seqs=4)
        assert eng.model.moe_ep and eng.model.layers[0]["w13_ep"].shape[0] == 4 // world
        outs = eng.generate(PROMPTS, SamplingParams(max_new_tokens=6))
        assert eng.model.ep_calls > 0
        q.put((rank, [o.token_ids for o in outs]))
    finally:
        dist.destroy_process_group()


def test_ep2_engine_matches_tp1():
    from distributed_llm_amd.engine.llm_engine import LLMEngine
    from distributed_llm_amd.engine.sampling import SamplingParams
    ref = [o.token_ids for o in LLMEngine("tiny-moe-test", device="cpu", kv_cache_gb=0.05, max_num_seqs=4)
           .generate(PROMPTS, SamplingParams(max_new_tokens=6))]
    res = _spawn(_engine_worker, 2)
    assert res[0] == res[1]
    for got, want in zip(res[0], ref):
        assert got[:3] == want[:3]
    same = sum(a == b for g, w in zip(res[0], ref) for a, b in zip(g, w))
    assert same >= 0.8 * sum(len(w) for w in ref)


def test_moe_router_cpu_matches_fp32_gate():
    """ops.moe_router off the GPU: fp32 projection + the same top-k / renormalised weights as
    ops.moe_gate (the kernel's semantics); rows are independent of the batch they arrive in."""
    from distributed_llm_amd import ops
    g = torch.Generator().manual_seed(0)
    x = torch.randn(9, 64, generator=g).bfloat16()
    wg = torch.randn(8, 64, generator=g).bfloat16()
    ids, w = ops.moe_router(x, wg, 2)
    ri, rw = ops.moe_gate(x.float() @ wg.float().t(), 2)
    assert torch.equal(ids, ri) and torch.allclose(w, rw)
    i3, w3 = ops.moe_router(x[:3], wg, 2)
    assert torch.equal(i3, ids[:3]) and torch.allclose(w3, w[:3])
