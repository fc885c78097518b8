"""Vocab-parallel sampler (ops.tp_candidates + ops.tp_sample, csrc/kernels/sampling.hip): the
per-shard ranked top-256 candidates, all-gathered and merged, draw exactly the token the
unsharded row sampler (ops.sample_rows) draws — greedy and top-k / top-p rows, ties broken by the
lowest global id.  CPU: the reference implementations; GPU: the HIP kernels against them."""
import pytest
import torch

from distributed_llm_amd import ops
from distributed_llm_amd.ops import reference as ref


def _case(S, V, seed):
    g = torch.Generator().manual_seed(seed)
    lg = (torch.randn(S, V, generator=g) * 3).to(torch.bfloat16)
    lg[0, 5] = lg[0, V - 3] = lg[0].max() + 1          # a tie at the top: lowest id wins
    temp = torch.tensor([0.0, 0.8, 1.3, 0.0, 0.7, 0.9][:S], dtype=torch.float32)
    top_p = torch.tensor([1.0, 0.9, 0.5, 1.0, 1.0, 0.95][:S], dtype=torch.float32)
    top_k = torch.tensor([0, 40, 0, 7, 256, 1][:S], dtype=torch.int32)
    return lg, temp, top_p, top_k


def _sharded(lg, tp, dev):
    V = lg.shape[1]
    sh = V // tp
    return torch.stack([ops.tp_candidates(lg[:, p * sh:(p + 1) * sh].contiguous().to(dev), p * sh) for p in range(tp)])


@pytest.mark.parametrize("tp", [1, 2, 4, 8])
def test_tp_sampler_matches_unsharded_reference(tp):
    S, V = 6, 4096
    lg, temp, top_p, top_k = _case(S, V, tp)
    seed = torch.tensor([1234], dtype=torch.int32)
    want = ref.sample_rows(lg, temp, top_p, top_k, 1234)
    got = ops.tp_sample(_sharded(lg, tp, "cpu"), temp, top_p, top_k, seed)
    assert got.tolist() == want.tolist()
    assert got[0].item() == 5


@pytest.mark.gpu
@pytest.mark.parametrize("tp", [1, 2, 4, 8])
@pytest.mark.parametrize("V", [32000, 128256])
def test_tp_sampler_kernels(tp, V):
    S = 6
    lg, temp, top_p, top_k = _case(S, V, V + tp)
    lg[3, 100:200] = float("nan")                        # NaN logits are never candidates
    dev = "cuda"
    seed = torch.tensor([99], dtype=torch.int32, device=dev)
    cands = _sharded(lg, tp, dev)
    sh = V // tp
    ref_c = torch.stack([ref.tp_candidates(lg[:, p * sh:(p + 1) * sh], p * sh) for p in range(tp)])
    assert torch.equal(cands.cpu(), ref_c)
    t, p_, k = temp.to(dev), top_p.to(dev), top_k.to(dev)
    got = ops.tp_sample(cands, t, p_, k, seed)
    want = ops.sample_rows(lg.to(dev), t, p_, k, seed)    # the unsharded HIP sampler
    assert got.tolist() == want.tolist()
    assert got.tolist() == ref.tp_sample(ref_c, temp, top_p, top_k, 99).tolist()
