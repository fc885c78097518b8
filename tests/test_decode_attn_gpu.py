"""Wave-per-unit decode attention (csrc/kernels/decode_attn.hip) against the fp32 reference:
static split grids and the persistent work list, GQA groups 1-16, head dims 64/96/128, padding
tiles, and never-written cache tails poisoned with NaN."""
import math

import numpy as np
import pytest
import torch

from distributed_llm_amd import ops
from distributed_llm_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _case(d, nq, nkv, ctxs, seed=0):
    g = torch.Generator().manual_seed(seed)
    nblocks = sum((c + 15) // 16 for c in ctxs) + 4
    kc = torch.full((nblocks, nkv, 16, d), float("nan"), dtype=torch.bfloat16)
    vc = torch.full((nblocks, nkv, d, 16), float("nan"), dtype=torch.bfloat16)
    perm = torch.randperm(nblocks - 1, generator=g) + 1
    maxb = max((c + 15) // 16 for c in ctxs)
    bt = torch.zeros(len(ctxs), maxb, dtype=torch.int32)
    k = 0
    for i, c in enumerate(ctxs):
        nb = (c + 15) // 16
        bt[i, :nb] = perm[k:k + nb].to(torch.int32)
        k += nb
        idx = bt[i, :nb].long()
        kk = torch.randn(nb * 16, nkv, d, generator=g).to(torch.bfloat16)
        vv = torch.randn(nb * 16, nkv, d, generator=g).to(torch.bfloat16)
        kk[c:] = float("nan")
        vv[c:] = float("nan")
        kc[idx] = kk.view(nb, 16, nkv, d).permute(0, 2, 1, 3)
        vc[idx] = vv.view(nb, 16, nkv, d).permute(0, 2, 3, 1)
    B = len(ctxs)
    q = torch.randn(B, nq, d, generator=g).to(torch.bfloat16)
    I = lambda x: torch.tensor(x, dtype=torch.int32)
    return q, kc, vc, bt, I(list(range(B))), I(ctxs)


def _want(q, kc, vc, bt, qs, cx, d):
    ql = torch.ones_like(cx)
    return ref.paged_attention(q, kc.nan_to_num(0.0), vc.nan_to_num(0.0), bt, qs, ql, cx, 1.0 / math.sqrt(d), True)


@pytest.mark.parametrize("d,nq,nkv", [(64, 32, 4), (128, 32, 8), (96, 32, 32), (128, 64, 4), (64, 16, 16)])
@pytest.mark.parametrize("splits", [1, 3, 8])
def test_decode_attention_static_grid(d, nq, nkv, splits):
    ctxs = [1, 15, 16, 17, 33, 100, 257, 1000, 2049]
    q, kc, vc, bt, qs, cx = _case(d, nq, nkv, ctxs, seed=d + splits)
    B = len(ctxs)
    order = np.argsort(-np.array(ctxs), kind="stable")
    tseq = torch.tensor(list(order) + [-1, -1], dtype=torch.int32)   # two padding tiles
    T = tseq.numel()
    C = lambda t: t.cuda()
    ws = (torch.empty(T * nkv * splits * 16 * d, device="cuda"), torch.empty(T * nkv * splits * 32, device="cuda"),
          torch.zeros(T * nkv + 2, dtype=torch.int32, device="cuda"))
    got = ops.decode_attention(C(q), C(kc), C(vc), C(bt), C(qs), C(cx), C(tseq), splits=splits, workspace=ws)
    assert torch.isfinite(got.float()).all()
    torch.testing.assert_close(got.cpu().float(), _want(q, kc, vc, bt, qs, cx, d).float(), atol=2e-2, rtol=2e-2)
    assert int(ws[2].abs().sum()) == 0          # tickets re-armed


@pytest.mark.parametrize("d,nq,nkv", [(64, 32, 4), (128, 32, 8)])
@pytest.mark.parametrize("target,min_chunk,grid", [(64, 256, 8), (4096, 64, 32), (512, 128, 1)])
def test_decode_attention_work_list(d, nq, nkv, target, min_chunk, grid):
    rng = np.random.default_rng(d + target)
    ctxs = rng.integers(1, 3000, size=37).tolist()
    q, kc, vc, bt, qs, cx = _case(d, nq, nkv, ctxs, seed=7)
    order = np.argsort(-np.array(ctxs), kind="stable")
    tseq = torch.tensor(order, dtype=torch.int32)
    max_splits = 16
    items = ops.decode_work_items(np.array(ctxs)[order], nkv, max_splits, target, min_chunk=min_chunk)
    B = len(ctxs)
    ws = (torch.empty(B * nkv * max_splits * 16 * d, device="cuda"),
          torch.empty(B * nkv * max_splits * 32, device="cuda"),
          torch.zeros(B * nkv + 2, dtype=torch.int32, device="cuda"))
    C = lambda t: t.cuda()
    for _ in range(2):   # second launch re-uses the re-armed tickets
        got = ops.decode_attention(C(q), C(kc), C(vc), C(bt), C(qs), C(cx), C(tseq), splits=max_splits, workspace=ws,
                                   items=torch.from_numpy(items).cuda(), grid_wgs=grid)
        torch.testing.assert_close(got.cpu().float(), _want(q, kc, vc, bt, qs, cx, d).float(), atol=2e-2, rtol=2e-2)


def test_engine_wave_decode_matches_default(monkeypatch):
    """The opt-in wave decode kernel gives the same greedy tokens as the default paged path
    through the whole engine (hipGraph decode, work list, splits)."""
    from distributed_llm_amd.engine.llm_engine import LLMEngine
    from distributed_llm_amd.engine.sampling import SamplingParams
    prompts = ["user: hello there", "user: " + "long context " * 60, "x", "user: explain recursion"]
    sp = SamplingParams(max_new_tokens=20)
    base = LLMEngine("tiny-llama-test", device="cuda", kv_cache_gb=0.5, max_num_seqs=8)
    a = [o.token_ids for o in base.generate(prompts, sp)]
    monkeypatch.setattr(LLMEngine, "DECODE_WAVE", True)
    wave = LLMEngine("tiny-llama-test", device="cuda", kv_cache_gb=0.5, max_num_seqs=8)
    b = [o.token_ids for o in wave.generate(prompts, sp)]
    # the two kernels sum in different orders (bf16 outputs can differ by an ulp), so a random-init
    # model may flip a near-tied argmax late in a sequence: require the first tokens to agree
    assert all(x[:8] == y[:8] for x, y in zip(a, b)), (a, b)
