"""Flash-style prefill attention (csrc/kernels/flash_prefill.hip) against the fp32 PyTorch
reference (ops.reference.paged_attention): ragged batches, cached prefixes (chunked prefill),
causal and bidirectional, GQA groups 1/4/8/16/32, head dims 64/96/128, scores whose running max
keeps rising (the online-softmax rescale path), and never-written cache tails poisoned with NaN
(they must not leak into the output)."""
import math

import pytest
import torch

from distributed_llm_amd import ops
from distributed_llm_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _case(d, nq, nkv, seqs, seed=0, rising=False):
    g = torch.Generator().manual_seed(seed)
    nblocks = sum((c + 15) // 16 for _, c in seqs) + 8
    kc = torch.full((nblocks, nkv, 16, d), float("nan"), dtype=torch.bfloat16)
    vc = torch.full((nblocks, nkv, d, 16), float("nan"), dtype=torch.bfloat16)
    perm = torch.randperm(nblocks - 1, generator=g) + 1
    maxb = max((c + 15) // 16 for _, c in seqs)
    bt = torch.zeros(len(seqs), maxb, dtype=torch.int32)
    k = 0
    for i, (_, c) in enumerate(seqs):
        nb = (c + 15) // 16
        bt[i, :nb] = perm[k:k + nb].to(torch.int32)
        k += nb
        for t in range(c):   # only the sequence's own tokens are written
            blk, off = int(bt[i, t // 16]), t % 16
            amp = (1.0 + t / 64.0) if rising else 1.0   # rising: the running max moves in late chunks
            kc[blk, :, off, :] = (amp * torch.randn(nkv, d, generator=g)).to(torch.bfloat16)
            vc[blk, :, :, off] = torch.randn(nkv, d, generator=g).to(torch.bfloat16)
    T = sum(q for q, _ in seqs)
    q = torch.randn(T, nq, d, generator=g).to(torch.bfloat16)
    qstart, acc = [], 0
    for ql, _ in seqs:
        qstart.append(acc)
        acc += ql
    I = lambda x: torch.tensor(x, dtype=torch.int32)
    return q, kc, vc, bt, I(qstart), I([s[0] for s in seqs]), I([s[1] for s in seqs])


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("d,nq,nkv", [(64, 32, 4), (128, 32, 8), (128, 8, 8), (64, 8, 1), (128, 64, 4), (64, 64, 2), (96, 32, 32)])
@pytest.mark.parametrize("rising", [False, True])
def test_flash_prefill_matches_fp32_reference(d, nq, nkv, causal, rising):
    seqs = [(300, 300), (37, 37), (200, 777), (129, 129), (1, 50), (16, 33)]
    q, kc, vc, bt, qs, ql, cx = _case(d, nq, nkv, seqs, seed=d + nq, rising=rising)
    ts, tt = ops.flash_tiles(ql.tolist(), nq // nkv)
    C = lambda t: t.cuda()
    got = ops.flash_attention(C(q), C(kc), C(vc), C(bt), C(qs), C(ql), C(cx), C(torch.tensor(ts, dtype=torch.int32)),
                              C(torch.tensor(tt, dtype=torch.int32)), causal=causal)
    want = ref.paged_attention(q, kc.nan_to_num(0.0), vc.nan_to_num(0.0), bt, qs, ql, cx, 1.0 / math.sqrt(d), causal)
    assert torch.isfinite(got.float()).all()
    torch.testing.assert_close(got.cpu().float(), want.float(), atol=2e-2, rtol=2e-2)


def test_flash_prefill_matches_paged_kernel_in_engine_shapes():
    """The flash path and the 16-row paged kernel agree on a TinyLlama-shaped prefill batch."""
    d, nq, nkv = 64, 32, 4
    seqs = [(1024, 1024), (513, 2048), (77, 77)]
    q, kc, vc, bt, qs, ql, cx = _case(d, nq, nkv, seqs, seed=5)
    C = lambda t: t.cuda()
    fts, ftt = ops.flash_tiles(ql.tolist(), nq // nkv)
    pts, ptt = ops.build_tiles(ql.tolist(), nq // nkv)
    I = lambda x: torch.tensor(x, dtype=torch.int32, device="cuda")
    kcz, vcz = C(kc.nan_to_num(0.0)), C(vc.nan_to_num(0.0))
    a = ops.flash_attention(C(q), kcz, vcz, C(bt), C(qs), C(ql), C(cx), I(fts), I(ftt))
    b = ops.paged_attention(C(q), kcz, vcz, C(bt), C(qs), C(ql), C(cx), I(pts), I(ptt))
    torch.testing.assert_close(a.float(), b.float(), atol=1e-2, rtol=1e-2)


@pytest.mark.parametrize("causal", [True, False])
def test_flash_prefill_past_one_block_table_window(causal):
    """Contexts past 16K keys (1024 block-table entries): the kernel re-stages its LDS block-table
    window every 16K keys instead of refusing.  Cached prefixes of 40K and 17K
    keys, a chunk of new queries each; scattered physical blocks."""
    d, nq, nkv = 64, 32, 4
    seqs = [(200, 40000), (64, 17000), (33, 16400)]
    g = torch.Generator().manual_seed(11)
    nbs = [(c + 15) // 16 for _, c in seqs]
    nblocks = sum(nbs) + 8
    kc = torch.full((nblocks, nkv, 16, d), float("nan"), dtype=torch.bfloat16)
    vc = torch.full((nblocks, nkv, d, 16), float("nan"), dtype=torch.bfloat16)
    perm = torch.randperm(nblocks - 1, generator=g) + 1
    bt = torch.zeros(len(seqs), max(nbs), dtype=torch.int32)
    k = 0
    for i, (_, c) in enumerate(seqs):
        blks = perm[k:k + nbs[i]]
        k += nbs[i]
        bt[i, :nbs[i]] = blks.to(torch.int32)
        kk = torch.randn(nbs[i] * 16, nkv, d, generator=g)
        vv = torch.randn(nbs[i] * 16, nkv, d, generator=g)
        kk[c:] = float("nan")            # never-written tail of the last block
        vv[c:] = float("nan")
        kc[blks] = kk.view(nbs[i], 16, nkv, d).permute(0, 2, 1, 3).to(torch.bfloat16)
        vc[blks] = vv.view(nbs[i], 16, nkv, d).permute(0, 2, 3, 1).to(torch.bfloat16)
    T = sum(q for q, _ in seqs)
    q = torch.randn(T, nq, d, generator=g).to(torch.bfloat16)
    I = lambda x: torch.tensor(x, dtype=torch.int32)
    qs = I([0, 200, 264])
    ql, cx = I([s[0] for s in seqs]), I([s[1] for s in seqs])
    ts, tt = ops.flash_tiles(ql.tolist(), nq // nkv)
    C = lambda t: t.cuda()
    assert ops.flash_supported(d, nq // nkv, bt.shape[1])
    got = ops.flash_attention(C(q), C(kc), C(vc), C(bt), C(qs), C(ql), C(cx), C(I(ts)), C(I(tt)), causal=causal)
    want = ref.paged_attention(q, kc.nan_to_num(0.0), vc.nan_to_num(0.0), bt, qs, ql, cx, 1.0 / math.sqrt(d), causal)
    assert torch.isfinite(got.float()).all()
    torch.testing.assert_close(got.cpu().float(), want.float(), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("splits", ["1", "2", "3", "16"])
@pytest.mark.parametrize("d,nq,nkv", [(64, 32, 4), (128, 32, 8), (96, 32, 32)])
@pytest.mark.parametrize("causal", [True, False])
def test_flash_prefill_split_kv_matches_reference(splits, d, nq, nkv, causal, monkeypatch):
    """Split-KV (short prompts leave the grid small): each (tile, kv head)'s key chunks dealt to
    1-16 workgroups, the last arriver combining their (m, l, O) partials; more splits than a short
    tile has chunks leaves the surplus workgroups empty.  Same fp32 reference, NaN-poisoned tails,
    rising maxima; the default (auto) split is covered by the tests above."""
    monkeypatch.setenv("DLLM_FLASH_SPLITS", splits)
    seqs = [(1024, 1024), (130, 1830), (1, 50), (40, 40)]
    q, kc, vc, bt, qs, ql, cx = _case(d, nq, nkv, seqs, seed=d + int(splits), rising=True)
    ts, tt = ops.flash_tiles(ql.tolist(), nq // nkv)
    C = lambda t: t.cuda()
    got = ops.flash_attention(C(q), C(kc), C(vc), C(bt), C(qs), C(ql), C(cx), C(torch.tensor(ts, dtype=torch.int32)),
                              C(torch.tensor(tt, dtype=torch.int32)), causal=causal)
    again = ops.flash_attention(C(q), C(kc), C(vc), C(bt), C(qs), C(ql), C(cx), C(torch.tensor(ts, dtype=torch.int32)),
                                C(torch.tensor(tt, dtype=torch.int32)), causal=causal)
    want = ref.paged_attention(q, kc.nan_to_num(0.0), vc.nan_to_num(0.0), bt, qs, ql, cx, 1.0 / math.sqrt(d), causal)
    assert torch.isfinite(got.float()).all()
    torch.testing.assert_close(got.cpu().float(), want.float(), atol=2e-2, rtol=2e-2)
    assert torch.equal(got, again)     # the tickets re-arm: a second launch combines the same way


def test_flash_split_choice():
    """Auto split-KV only for small grids over long contexts (measured slower on short ones)."""
    assert ops.flash_splits(1000, 16384) == 1 and ops.flash_splits(256, 16384) == 1
    assert ops.flash_splits(128, 1024) == 1 and ops.flash_splits(20, 0) == 1
    assert ops.flash_splits(128, 16384) == 4 and ops.flash_splits(20, 16384) == 8 and ops.flash_splits(20, 4096) == 2
