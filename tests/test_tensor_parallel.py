"""Tensor parallelism on CPU (gloo, world_size 2): a TP=2 engine must generate exactly the tokens of
the TP=1 engine (same seed, greedy) up to late bf16 near-ties, dense and MoE; distributed arg-max /
top-k helpers agree."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


PROMPTS = ["user: hello there", "user: explain paged attention step by step", "x" * 70]


def _worker(rank, world, port, model, q, env=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    os.environ.update(env or {})
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from distributed_llm_amd.engine.llm_engine import LLMEngine
        from distributed_llm_amd.engine.sampling import SamplingParams
        from distributed_llm_amd.parallel.comm import make_tp_groups
        par = make_tp_groups(world)
        eng = LLMEngine(model, device="cpu", par=par, kv_cache_gb=0.05, max_num_seqs=4)
        sp = (SamplingParams(max_new_tokens=6, temperature=0.9, top_k=40, top_p=0.95)
              if os.environ.get("TP_TEST_SAMPLED") == "1" else SamplingParams(max_new_tokens=6))
        outs = eng.generate(PROMPTS, sp)
        q.put((rank, [o.token_ids for o in outs], eng.model.par.use_sp(64)))
    finally:
        dist.destroy_process_group()


def _run_tp(model, world=2, env=None, want_sp=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, model, q, env)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in procs]
    assert all(sp == want_sp for _, _, sp in got)
    res = {r: toks for r, toks, _ in got}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("model", ["tiny-llama-test", "tiny-moe-test"])
def test_tp2_matches_tp1(model):
    from distributed_llm_amd.engine.llm_engine import LLMEngine
    from distributed_llm_amd.engine.sampling import SamplingParams
    ref = [o.token_ids for o in LLMEngine(model, device="cpu", kv_cache_gb=0.05, max_num_seqs=4)
           .generate(PROMPTS, SamplingParams(max_new_tokens=6))]
    res = _run_tp(model)
    # TP ranks must agree bit-for-bit (they run in lockstep on all-reduced activations) ...
    assert res[0] == res[1]
    # ... and follow TP=1 greedy decoding; bf16 partial sums are rounded before the all-reduce,
    # so a late near-tie may flip — require the first tokens exactly and >= 80 % overall.
    for got, want in zip(res[0], ref):
        assert got[:3] == want[:3]
    same = sum(a == b for g, w in zip(res[0], ref) for a, b in zip(g, w))
    assert same >= 0.8 * sum(len(w) for w in ref)


def test_tp2_sampled_ranks_agree_and_follow_tp1():
    """Sampling under TP (LlamaModel.sample: merged per-shard top-256 candidates + the fused
    sampler with a shared seed): both ranks draw the same tokens, and the first draw matches TP=1
    (same exact top-k set and the same counter-based uniform)."""
    from distributed_llm_amd.engine.llm_engine import LLMEngine
    from distributed_llm_amd.engine.sampling import SamplingParams
    sp = SamplingParams(max_new_tokens=6, temperature=0.9, top_k=40, top_p=0.95)
    ref = [o.token_ids for o in LLMEngine("tiny-llama-test", device="cpu", kv_cache_gb=0.05, max_num_seqs=4)
           .generate(PROMPTS, sp)]
    res = _run_tp("tiny-llama-test", env={"TP_TEST_SAMPLED": "1"})
    assert res[0] == res[1]
    assert [g[0] for g in res[0]] == [w[0] for w in ref]


@pytest.mark.parametrize("model", ["tiny-llama-test", "tiny-moe-test"])
def test_sequence_parallel_prefill_matches_plain_tp(model):
    """Megatron-SP prefill (reduce-scatter / sharded norms / all-gather) must reproduce the plain
    TP=2 engine: prefill batches here are >= 2 tokens, so every prefill step takes the SP path."""
    plain = _run_tp(model)
    sp = _run_tp(model, env={"DLLM_SEQ_PARALLEL": "1", "DLLM_SP_MIN_TOKENS": "2"}, want_sp=True)
    assert sp[0] == sp[1]
    for got, want in zip(sp[0], plain[0]):
        assert got[:3] == want[:3]
    same = sum(a == b for g, w in zip(sp[0], plain[0]) for a, b in zip(g, w))
    assert same >= 0.8 * sum(len(w) for w in plain[0])


def test_shard_range_validation():
    from distributed_llm_amd.parallel.comm import shard_range
    assert shard_range(8, 1, 2) == slice(4, 8)
    with pytest.raises(ValueError):
        shard_range(7, 0, 2)
