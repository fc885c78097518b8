"""Numerics of every HIP kernel vs the plain-PyTorch f32 reference (ops.reference)."""
import math

import pytest
import numpy as np
import torch

from distributed_llm_amd import ops
from distributed_llm_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _native():
    assert ops.native_available(), "HIP extension must be built for GPU tests"


def bf(*s, scale=1.0):
    return (torch.randn(*s, device=DEV) * scale).to(torch.bfloat16)


@pytest.mark.parametrize("H", [384, 2048, 3072, 4096, 8192])
@pytest.mark.parametrize("with_res", [False, True])
def test_rms_norm(H, with_res):
    torch.manual_seed(0)
    x, w = bf(37, H), bf(H)
    r1 = bf(37, H) if with_res else None
    r2 = r1.clone() if with_res else None
    y = ops.rms_norm(x, w, 1e-5, residual=r1)
    yr = ref.rms_norm(x, w, 1e-5, residual=r2)
    torch.testing.assert_close(y.float(), yr.float(), atol=3e-2, rtol=2e-2)
    if with_res:
        torch.testing.assert_close(r1, r2, atol=0, rtol=0)


def test_layer_norm():
    torch.manual_seed(1)
    x, w, b, r = bf(50, 384), bf(384), bf(384), bf(50, 384)
    r2 = r.clone()
    y = ops.layer_norm(x, w, b, 1e-12, residual=r)
    yr = ref.layer_norm(x, w, b, 1e-12, residual=r2)
    torch.testing.assert_close(y.float(), yr.float(), atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("nq,nkv,d", [(32, 4, 64), (32, 8, 128), (32, 32, 96)])
def test_rope_and_cache(nq, nkv, d):
    torch.manual_seed(2)
    T, NB = 29, 8
    qkv = bf(T, (nq + 2 * nkv) * d)
    pos = torch.randint(0, 500, (T,), device=DEV, dtype=torch.int32)
    perm = torch.randperm(NB * 16, device=DEV)[:T].to(torch.int32)
    perm[3] = -1
    cs = ops.rope_cos_sin(1024, d, 10000.0, DEV)
    kc, vc = torch.zeros(NB, nkv, 16, d, dtype=torch.bfloat16, device=DEV), torch.zeros(NB, nkv, d, 16, dtype=torch.bfloat16, device=DEV)
    kc2, vc2 = kc.clone(), vc.clone()
    q = ops.rope_and_cache(qkv, pos, cs, perm, kc, vc, nq, nkv, d)
    q2 = ref.rope_and_cache(qkv, pos, cs, perm, kc2, vc2, nq, nkv, d)
    torch.testing.assert_close(q.float(), q2.float(), atol=2e-2, rtol=1e-2)
    torch.testing.assert_close(kc.float(), kc2.float(), atol=2e-2, rtol=1e-2)
    torch.testing.assert_close(vc, vc2, atol=0, rtol=0)


def _attn_case(nq, nkv, d, seqs, NB=64, spike=False, seed=3):
    torch.manual_seed(seed)
    kc, vc = bf(NB, nkv, 16, d), bf(NB, nkv, d, 16)
    S = len(seqs)
    maxb = max((c + 15) // 16 for _, c in seqs)
    bt = torch.zeros(S, maxb, dtype=torch.int32)
    perm = torch.randperm(NB)
    k = 0
    for s, (_, c) in enumerate(seqs):
        nb = (c + 15) // 16
        bt[s, :nb] = perm[k:k + nb]
        k += nb
    assert k <= NB
    T = sum(q for q, _ in seqs)
    q = bf(T, nq, d)
    if spike:  # force online-softmax rescales: one huge key late in each sequence
        for s, (_, c) in enumerate(seqs):
            key = c - 3
            blk, off = int(bt[s, key // 16]), key % 16
            kc[blk, :, off, :] = 8.0
        q = q.abs()
    qstart, qlen, ctx = [], [], []
    t = 0
    for ql, c in seqs:
        qstart.append(t); qlen.append(ql); ctx.append(c); t += ql
    ts, tt = ops.build_tiles(qlen, nq // nkv)
    I = lambda x: torch.tensor(x, dtype=torch.int32, device=DEV)
    return q, kc, vc, bt.to(DEV), I(qstart), I(qlen), I(ctx), I(ts), I(tt)


@pytest.mark.parametrize("nq,nkv,d", [(32, 4, 64), (32, 8, 64), (32, 8, 128), (32, 32, 96), (64, 8, 128), (16, 16, 64)])
@pytest.mark.parametrize("splits", [1, 4])
def test_paged_attention_mixed(nq, nkv, d, splits):
    # decode rows (qlen 1), prefix-cached prefill (qlen < ctx), fresh prefill (qlen == ctx), ragged sizes
    seqs = [(1, 1), (1, 17), (1, 300), (5, 40), (33, 33), (7, 129), (1, 64), (16, 16)]
    q, kc, vc, bt, qs, ql, cx, ts, tt = _attn_case(nq, nkv, d, seqs, NB=96)
    scale = 1 / math.sqrt(d)
    o = ops.paged_attention(q, kc, vc, bt, qs, ql, cx, ts, tt, scale=scale, splits=splits)
    o2 = ref.paged_attention(q, kc, vc, bt, qs, ql, cx, scale)
    torch.testing.assert_close(o.float(), o2.float(), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("splits", [1, 3])
def test_paged_attention_rescale_branch(splits):
    seqs = [(1, 200), (9, 150), (1, 1000)]
    q, kc, vc, bt, qs, ql, cx, ts, tt = _attn_case(32, 8, 128, seqs, NB=96, spike=True)
    o = ops.paged_attention(q, kc, vc, bt, qs, ql, cx, ts, tt, splits=splits)
    o2 = ref.paged_attention(q, kc, vc, bt, qs, ql, cx, 1 / math.sqrt(128))
    torch.testing.assert_close(o.float(), o2.float(), atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("split_len,z", [(32, 8), (64, 4), (256, 8), (4096, 4)])
def test_paged_attention_dynamic_split(split_len, z):
    """Dynamic split-K: each tile takes ceil(keys / split_len) of the z splits (decode path), mixed
    with prefill tiles and an empty padding tile; repeated launches re-use the ticket counters."""
    seqs = [(1, 1), (1, 17), (1, 300), (1, 1000), (5, 40), (1, 64), (9, 150)]
    q, kc, vc, bt, qs, ql, cx, ts, tt = _attn_case(32, 8, 128, seqs, NB=128, spike=True)
    ts = torch.cat([ts, torch.tensor([-1], dtype=torch.int32, device=DEV)])   # padding tile
    tt = torch.cat([tt, torch.tensor([0], dtype=torch.int32, device=DEV)])
    nt, nkv, d = ts.numel(), kc.shape[1], 128
    ws = (torch.empty(nt * nkv * z * 16 * d, device=DEV), torch.empty(nt * nkv * z * 16 * 2, device=DEV),
          torch.zeros(nt * nkv, dtype=torch.int32, device=DEV))
    sl = torch.tensor([split_len], dtype=torch.int32, device=DEV)
    o2 = ref.paged_attention(q, kc, vc, bt, qs, ql, cx, 1 / math.sqrt(d))
    for _ in range(3):
        o = ops.paged_attention(q, kc, vc, bt, qs, ql, cx, ts, tt, splits=z, workspace=ws, split_len=sl)
        torch.testing.assert_close(o.float(), o2.float(), atol=3e-2, rtol=3e-2)
    assert int(ws[2].abs().sum()) == 0   # every ticket counter re-armed


@pytest.mark.parametrize("nq,nkv,d", [(32, 4, 64), (32, 8, 128), (64, 8, 128)])
@pytest.mark.parametrize("grid,target,min_chunk", [(1, 4, 32), (7, 16, 32), (64, 256, 256), (512, 2048, 256)])
@pytest.mark.parametrize("ext", [False, True])
def test_paged_attention_worklist(nq, nkv, d, grid, target, min_chunk, ext):
    """Persistent decode attention: a fixed grid walks a host-built list of (tile, kv head, split)
    units (1..16 splits per tile, longest first); repeated launches re-use the ticket counters.
    ``ext``: the extended list whose units carry (sequence, query row, context) themselves."""
    ctxs = [1000, 1, 17, 300, 64, 2047, 33, 512, 129, 5]
    seqs = [(1, c) for c in ctxs]
    q, kc, vc, bt, qs, ql, cx, ts, tt = _attn_case(nq, nkv, d, seqs, NB=320, spike=True)
    order = np.argsort(-np.array(ctxs), kind="stable")
    ts = torch.tensor(order.astype(np.int32), device=DEV)       # tile i -> sequence order[i]
    tt = torch.zeros_like(ts)
    z = 16
    nt = ts.numel()
    ws = (torch.empty(nt * nkv * z * 16 * d, device=DEV), torch.empty(nt * nkv * z * 16 * 2, device=DEV),
          torch.zeros(nt * nkv + 2, dtype=torch.int32, device=DEV))
    if ext:
        items = ops.decode_work_items(np.array(ctxs)[order], nkv, z, target, min_chunk=min_chunk, seq=order,
                                      qstart=qs.cpu().numpy()[order])
        n = -int(items[0])
        w = items[4:4 + 4 * n].reshape(n, 4)
    else:
        items = ops.decode_work_items(np.array(ctxs)[order], nkv, z, target, min_chunk=min_chunk)
        n = int(items[0])
        w = items[1:1 + 2 * n].reshape(n, 2)
    assert ((w[:, 1] & 0xFF) < (w[:, 1] >> 8)).all() and (w[:, 1] >> 8).max() <= z
    it = torch.tensor(items, device=DEV)
    o2 = ref.paged_attention(q, kc, vc, bt, qs, ql, cx, 1 / math.sqrt(d))
    for _ in range(3):
        o = ops.paged_attention(q, kc, vc, bt, qs, ql, cx, ts, tt, splits=z, workspace=ws, items=it,
                                grid_items=grid)
        torch.testing.assert_close(o.float(), o2.float(), atol=3e-2, rtol=3e-2)
    assert int(ws[2].abs().sum()) == 0


@pytest.mark.parametrize("nq,nkv,d", [(32, 4, 64), (32, 8, 64), (16, 16, 64)])
@pytest.mark.parametrize("ext,grid", [(True, 7), (True, 512), (False, 64)])
def test_paged_attention_decode_writes_newest_v(nq, nkv, d, ext, grid):
    """Decode hand-over (AttnArgs.v_new): each sequence's newest V arrives row-major and its V^T
    cache slot holds garbage (NaN); the unit that owns the newest key must write it into the cache
    and attend with it.  Output equals the reference with V written first, the cache slot holds the
    new V afterwards, and a repeated launch (now reading the written cache) agrees."""
    ctxs = [1000, 1, 17, 300, 64, 2047, 33, 512, 129, 5, 16, 32]
    seqs = [(1, c) for c in ctxs]
    q, kc, vc, bt, qs, ql, cx, ts, tt = _attn_case(nq, nkv, d, seqs, NB=320)
    T = q.shape[0]
    vnew = (torch.randn(T, nkv * d, device=DEV) * 2).to(torch.bfloat16)
    vc_ref = vc.clone()
    ref.write_newest_v(vnew, vc_ref, bt, qs, cx)
    for s_, c in enumerate(ctxs):          # poison the newest slot in the cache the kernel reads
        key = c - 1
        vc[int(bt[s_, key // 16]), :, :, key % 16] = float("nan")
    order = np.argsort(-np.array(ctxs), kind="stable")
    ts = torch.tensor(order.astype(np.int32), device=DEV)
    tt = torch.zeros_like(ts)
    z, nt = 16, ts.numel()
    ws = (torch.empty(nt * nkv * z * 16 * d, device=DEV), torch.empty(nt * nkv * z * 16 * 2, device=DEV),
          torch.zeros(nt * nkv + 2, dtype=torch.int32, device=DEV))
    if ext:
        items = ops.decode_work_items(np.array(ctxs)[order], nkv, z, 256, min_chunk=32, seq=order,
                                      qstart=qs.cpu().numpy()[order])
    else:
        items = ops.decode_work_items(np.array(ctxs)[order], nkv, z, 256, min_chunk=32)
    it = torch.tensor(items, device=DEV)
    o2 = ref.paged_attention(q, kc.clone(), vc_ref, bt, qs, ql, cx, 1 / math.sqrt(d))
    o = ops.paged_attention(q, kc, vc, bt, qs, ql, cx, ts, tt, splits=z, workspace=ws, items=it, grid_items=grid,
                            v_new=vnew)
    torch.testing.assert_close(o.float(), o2.float(), atol=3e-2, rtol=3e-2)
    assert torch.equal(vc, vc_ref)          # every newest slot written, nothing else touched
    o3 = ops.paged_attention(q, kc, vc, bt, qs, ql, cx, ts, tt, splits=z, workspace=ws, items=it, grid_items=grid)
    torch.testing.assert_close(o3.float(), o2.float(), atol=3e-2, rtol=3e-2)


def test_paged_attention_newest_v_refused_for_wide_heads():
    """The v_new patch is built for head_dim 64 only; d = 128 must fail loudly, not skip the write."""
    q, kc, vc, bt, qs, ql, cx, ts, tt = _attn_case(32, 8, 128, [(1, 40), (1, 7)], NB=16)
    items = torch.tensor(ops.decode_work_items(np.array([40, 7]), 8, 4, 256, min_chunk=32), device=DEV)
    ws = (torch.empty(2 * 8 * 4 * 16 * 128, device=DEV), torch.empty(2 * 8 * 4 * 16 * 2, device=DEV),
          torch.zeros(2 * 8 + 2, dtype=torch.int32, device=DEV))
    with pytest.raises(RuntimeError):
        ops.paged_attention(q, kc, vc, bt, qs, ql, cx, ts, tt, splits=4, workspace=ws, items=items, grid_items=64,
                            v_new=torch.zeros(2, 8 * 128, dtype=torch.bfloat16, device=DEV))


def test_paged_attention_bidirectional():
    seqs = [(20, 20), (7, 7)]
    q, kc, vc, bt, qs, ql, cx, ts, tt = _attn_case(16, 16, 64, seqs)
    o = ops.paged_attention(q, kc, vc, bt, qs, ql, cx, ts, tt, causal=False)
    o2 = ref.paged_attention(q, kc, vc, bt, qs, ql, cx, 1 / 8.0, causal=False)
    torch.testing.assert_close(o.float(), o2.float(), atol=2e-2, rtol=2e-2)


def test_silu_mul_gelu():
    torch.manual_seed(4)
    gu = bf(19, 2 * 5632)
    torch.testing.assert_close(ops.silu_mul(gu).float(), ref.silu_mul(gu).float(), atol=2e-2, rtol=2e-2)
    x = bf(7, 1536)
    torch.testing.assert_close(ops.gelu(x).float(), ref.gelu(x).float(), atol=2e-2, rtol=2e-2)


def test_mean_pool_l2():
    torch.manual_seed(5)
    x = bf(6, 33, 384)
    lens = torch.tensor([1, 5, 33, 2, 17, 33], dtype=torch.int32, device=DEV)
    torch.testing.assert_close(ops.mean_pool_l2(x, lens), ref.mean_pool_l2(x, lens), atol=1e-3, rtol=1e-3)


def test_moe_gate():
    torch.manual_seed(6)
    lg = torch.randn(300, 8, device=DEV)
    ids, w = ops.moe_gate(lg, 2)
    ids2, w2 = ref.moe_gate(lg, 2)
    assert torch.equal(ids.long(), ids2.long())
    torch.testing.assert_close(w, w2, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("V", [32000, 32064, 128256, 1001])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_argmax(V, dtype):
    torch.manual_seed(7)
    Vp = (V + 15) // 8 * 8  # strided rows, row stride kept 16-B aligned
    lg = torch.randn(9, Vp, device=DEV).to(dtype)[:, :V]
    lg[3, 17] = 100.0
    a = ops.argmax(lg)
    assert torch.equal(a.long(), torch.argmax(lg.float(), -1))


def test_sample_top_p():
    torch.manual_seed(8)
    B, K = 64, 40
    vals = torch.sort(torch.randn(B, K, device=DEV) * 3, dim=-1, descending=True).values
    idx = torch.randint(0, 32000, (B, K), device=DEV)
    temp = torch.rand(B, device=DEV) + 0.3
    top_p = torch.rand(B, device=DEV) * 0.9 + 0.1
    u = torch.rand(B, device=DEV)
    a = ops.sample_top_p(vals, idx, temp, top_p, u)
    b = ref.sample_top_p(vals, idx, temp, top_p, u)
    # identical except for float ties at CDF boundaries
    assert (a.long() == b.long()).float().mean() > 0.95


@pytest.mark.parametrize("V", [32000, 1000, 37])
def test_sample_rows_matches_reference(V):
    torch.manual_seed(9)
    B = 48
    Vp = (V + 7) // 8 * 8        # rows stay 16-B aligned; V = 37 exercises the scalar tail
    lg = (torch.randn(B, Vp, device=DEV) * 2.0).to(torch.bfloat16)[:, :V]
    temp = torch.where(torch.arange(B, device=DEV) % 4 == 0, torch.zeros(B, device=DEV),
                       torch.rand(B, device=DEV) + 0.3)
    top_p = torch.rand(B, device=DEV) * 0.9 + 0.1
    top_k = torch.tensor([[0, 1, 5, 40][i % 4] if i % 3 else 256 for i in range(B)], dtype=torch.int32, device=DEV)
    seed = torch.tensor([12345], dtype=torch.int32, device=DEV)
    a = ops.sample_rows(lg, temp, top_p, top_k, seed).cpu()
    b = ref.sample_rows(lg.cpu(), temp.cpu(), top_p.cpu(), top_k.cpu(), 12345)
    greedy = (temp.cpu() <= 0)
    assert torch.equal(a[greedy], b[greedy])
    assert torch.equal(a[greedy].long(), lg.float().argmax(-1).cpu()[greedy])
    # sampled rows: identical except for float rounding at CDF boundaries; always inside the top-k
    assert (a == b).float().mean() > 0.95
    for r in range(B):
        k = int(top_k[r]) if 0 < int(top_k[r]) <= 256 else 256
        kth = torch.topk(lg[r].float(), min(k, V)).values[-1]
        assert lg[r, int(a[r])].float() >= kth


def test_sample_rows_crowded_ties_and_distribution():
    # heavy ties at the top (exercises the exact-threshold pass and candidate-list overflow)
    B, V = 8, 32000
    lg = torch.randint(0, 4, (B, V), device=DEV).to(torch.bfloat16)
    p = lambda x: torch.full((B,), x, device=DEV)
    a = ops.sample_rows(lg, p(1.0), p(0.9), torch.full((B,), 40, dtype=torch.int32, device=DEV),
                        torch.tensor([3], dtype=torch.int32, device=DEV))
    assert bool((lg.gather(1, a.long()[:, None]).float() == 3.0).all())
    # many rows of the same small-vocab logits: empirical frequencies follow softmax(logits / t)
    B, V, t = 8192, 8, 0.7
    base = torch.tensor([2.0, 1.5, 1.0, 0.5, 0.0, -0.5, -1.0, -3.0], device=DEV)
    lg = base.to(torch.bfloat16).expand(B, V).contiguous()
    pick = ops.sample_rows(lg, p(t)[:1].expand(B).contiguous(), torch.ones(B, device=DEV),
                           torch.zeros(B, dtype=torch.int32, device=DEV),
                           torch.tensor([99], dtype=torch.int32, device=DEV))
    freq = torch.bincount(pick.long(), minlength=V).float() / B
    want = torch.softmax(base.to(torch.bfloat16).float() / t, 0)
    assert (freq - want).abs().max() < 0.02


def test_sample_rows_tie_flood_keeps_strictly_better_candidates():
    """more ties AT the top-k threshold than the candidate list holds must never push
    out a strictly better logit.  10 clear winners sit at the END of the vocab (appended last by
    the scan) behind 3000 exact ties; with top_p = 0.5 the nucleus lies inside the winners."""
    B, V = 64, 32000
    lg = torch.full((B, V), -4.0, device=DEV)
    lg[:, 1000:4000] = 1.0
    lg[:, V - 10:] = 5.0
    lg = lg.to(torch.bfloat16)
    p = lambda x: torch.full((B,), x, device=DEV)
    a = ops.sample_rows(lg, p(1.0), p(0.5), torch.full((B,), 50, dtype=torch.int32, device=DEV),
                        torch.tensor([17], dtype=torch.int32, device=DEV)).cpu()
    assert bool((a >= V - 10).all()), a


@pytest.mark.parametrize("B,V", [(1, 32000), (3, 32000), (8, 128256), (2, 32005), (5, 8200)])
def test_sample_split_matches_one_workgroup_per_row(B, V):
    """Small batches run the split-vocab sampler (P shards per row, last arriver merges): the token
    of every row equals the one-workgroup-per-row kernel's, greedy and sampled, any top_k."""
    P = max(2, min(8, V // ops.SAMPLE_SPLIT_SHARD))
    split = lambda *a, **kw: ops.sample_rows(*a, shards=P, **kw)
    torch.manual_seed(B * 7 + V)
    Vp = (V + 7) // 8 * 8
    ext = ops._native(torch.empty(1, device=DEV))
    for trial in range(4):
        lg = (torch.randn(B, Vp, device=DEV) * 3.0).to(torch.bfloat16)[:, :V]
        temp = torch.where(torch.arange(B, device=DEV) % 3 == trial % 3, torch.zeros(B, device=DEV),
                           torch.rand(B, device=DEV) + 0.3)
        top_p = torch.rand(B, device=DEV) * 0.9 + 0.1
        top_k = torch.tensor([[0, 1, 5, 40, 256, 300][(i + trial) % 6] for i in range(B)], dtype=torch.int32,
                             device=DEV)
        seed = torch.tensor([1000 + trial], dtype=torch.int32, device=DEV)
        a = split(lg, temp, top_p, top_k, seed)
        b = torch.empty(B, dtype=torch.int32, device=DEV)
        ext.sample_rows(lg, temp, top_p, top_k, seed, b)
        assert torch.equal(a.cpu(), b.cpu()), (trial, a, b)
    # the tie flood of the test above on the split path: strictly better logits are never dropped
    lg = torch.full((B, V), -4.0, device=DEV)
    lg[:, 1000:4000] = 1.0
    lg[:, V - 10:] = 5.0
    lg = torch.cat([lg, torch.zeros(B, Vp - V, device=DEV)], 1).to(torch.bfloat16)[:, :V]
    p = lambda x: torch.full((B,), x, device=DEV)
    a = split(lg, p(1.0), p(0.5), torch.full((B,), 50, dtype=torch.int32, device=DEV),
                        torch.tensor([17], dtype=torch.int32, device=DEV)).cpu()
    assert bool((a >= V - 10).all()), a
    # a NaN row yields a real token, as the unsplit kernel does
    lg[0] = float("nan")     # in place: keeps the padded (16-B aligned) row stride
    a = split(lg, p(0.0), p(1.0), torch.zeros(B, dtype=torch.int32, device=DEV),
                        torch.tensor([1], dtype=torch.int32, device=DEV))
    b = torch.empty(B, dtype=torch.int32, device=DEV)
    ext.sample_rows(lg, p(0.0), p(1.0), torch.zeros(B, dtype=torch.int32, device=DEV),
                    torch.tensor([1], dtype=torch.int32, device=DEV), b)
    assert torch.equal(a.cpu(), b.cpu())


def test_sample_split_in_a_graph():
    """The split sampler replays in a captured graph (its ticket counters re-arm themselves)."""
    B, V = 2, 128256
    assert ops.sample_split_shards(B, V) > 1 and ops.sample_split_shards(B, 32000) == 1
    lg = (torch.randn(B, V, device=DEV) * 3.0).to(torch.bfloat16)
    temp, top_p = torch.full((B,), 0.8, device=DEV), torch.full((B,), 0.9, device=DEV)
    top_k = torch.full((B,), 40, dtype=torch.int32, device=DEV)
    seed = torch.tensor([5], dtype=torch.int32, device=DEV)
    out = torch.empty(B, dtype=torch.int32, device=DEV)
    ops.sample_rows(lg, temp, top_p, top_k, seed, out=out)     # workspace created outside capture
    want = out.clone()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            ops.sample_rows(lg, temp, top_p, top_k, seed, out=out)
    for _ in range(3):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, want)


def test_cosine_kernels():
    torch.manual_seed(9)
    q, c = torch.randn(5, 384, device=DEV), torch.randn(7, 384, device=DEV)
    torch.testing.assert_close(ops.cosine_scores(q, c), ref.cosine_scores(q, c), atol=1e-5, rtol=1e-4)
    N = 5000
    table = torch.randn(N, 384, device=DEV)
    qv = table[1234] + 0.05 * torch.randn(384, device=DEV)
    norms = table.norm(dim=-1)
    ctx = torch.randint(0, 3, (N,), device=DEV, dtype=torch.int32)
    ctx[1234] = 2
    r, s = ops.masked_cosine_argmax(qv, table, norms, ctx, 2, 0.85)
    r2, s2 = ref.masked_cosine_argmax(qv, table, norms, ctx, 2, 0.85)
    assert r == r2 == 1234 and abs(s - s2) < 1e-4
    r, s = ops.masked_cosine_argmax(qv, table, norms, ctx, 1, 0.85)
    assert r == -1


@pytest.mark.parametrize("M", [1, 5, 16, 33, 64, 100, 128])
@pytest.mark.parametrize("N,K", [(2560, 2048), (2048, 5632), (200, 96)])
@pytest.mark.parametrize("ntw,splits", [(1, 1), (2, 4), (4, 8), (1, 16)])
def test_skinny_gemm(M, N, K, ntw, splits):
    from distributed_llm_amd.ops import gemm
    kind = "skinny"
    if M > 64 and ntw == 4:
        pytest.skip("unsupported tile")
    torch.manual_seed(10)
    x, w = bf(M, K, scale=0.5), bf(N, K, scale=0.05)
    y = gemm._run_plan((kind, ntw, splits), x, w, False, None)
    yr = (x.float() @ w.float().T)
    torch.testing.assert_close(y.float(), yr, atol=2e-2, rtol=2e-2)
    # repeated launches reuse the re-armed counters
    y2 = gemm._run_plan((kind, ntw, splits), x, w, False, None)
    assert torch.equal(y, y2)


@pytest.mark.parametrize("M", [1, 64, 128])
def test_skinny_gemm_swiglu(M):
    from distributed_llm_amd.ops import gemm
    kind = "skinny"
    torch.manual_seed(11)
    I, H = 1024, 512
    gu, w = bf(M, 2 * I), bf(H, I, scale=0.05)
    y = gemm._run_plan((kind, 2 if M <= 64 else 1, 4), gu, w, True, None)
    yr = ref.silu_mul(gu).float() @ w.float().T
    torch.testing.assert_close(y.float(), yr, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("T,H,I,E,k", [(1, 128, 64, 4, 2), (7, 256, 96, 8, 2), (64, 512, 256, 8, 2),
                                       (300, 256, 128, 8, 2), (33, 128, 160, 4, 1), (16, 4096, 1792, 8, 2)])
def test_moe_ffn(T, H, I, E, k):
    """Grouped MoE FFN (routing + gathered GEMMs + SwiGLU + combine) vs the torch fp32 reference."""
    g = torch.Generator(device="cuda").manual_seed(T * 31 + E)
    x = (torch.randn(T, H, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
    w13 = (torch.randn(E, 2 * I, H, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    w2 = (torch.randn(E, H, I, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    logits = torch.randn(T, E, device="cuda", generator=g)
    ids, w = ops.moe_gate(logits, k)
    got = ops.moe_ffn(x, ids, w, w13, w2).float()
    want = ref.moe_ffn(x, ids, w, w13, w2).float()
    err = (got - want).abs().max().item()
    assert err <= 2e-2 * max(1.0, want.abs().max().item()), err


_MOE_PLANS = [(64, 128, 3, 1, 4, 64, 3, 1, 4), (128, 128, 3, 1, 8, 128, 3, 1, 8), (64, 64, 2, 2, 4, 128, 2, 1, 4),
              (256, 256, 2, 1, 8, 128, 3, 1, 8)]


@pytest.mark.parametrize("plan", _MOE_PLANS)
@pytest.mark.parametrize("T,H,I,E,k", [(1, 128, 64, 4, 2), (7, 256, 192, 8, 2), (300, 256, 128, 8, 2),
                                       (33, 128, 320, 4, 1), (16, 4096, 1792, 8, 2), (515, 512, 256, 8, 2)])
def test_moe_ffn_grouped_tgemm(T, H, I, E, k, plan):
    """MoE on the grouped LDS-tiled GEMM (moe_ffn_tg, interleaved gate/up) vs the fp32 reference."""
    from distributed_llm_amd.models.llama import gate_up_order
    g = torch.Generator(device="cuda").manual_seed(T * 7 + I)
    x = (torch.randn(T, H, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
    w13 = (torch.randn(E, 2 * I, H, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    w2 = (torch.randn(E, H, I, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    ids, w = ops.moe_gate(torch.randn(T, E, device="cuda", generator=g), k)
    w13i = w13.index_select(1, gate_up_order(I).cuda()).contiguous()
    got = ops.moe_ffn_tg(x, ids, w, w13i, w2, plan).float()
    want = ref.moe_ffn(x, ids, w, w13, w2).float()
    err = (got - want).abs().max().item()
    assert err <= 2e-2 * max(1.0, want.abs().max().item()), err


@pytest.mark.parametrize("H,E,k", [(256, 4, 2), (4096, 8, 2), (2048, 16, 4), (8192, 64, 8)])
def test_moe_router_matches_fp32_and_is_batch_invariant(H, E, k):
    """Fused router (fp32 projection + top-k) vs fp32 logits -> ref.moe_gate; a token's routing is
    bitwise the same whether it runs alone, in a small batch or in a padded one."""
    T = 37
    g = torch.Generator(device="cuda").manual_seed(H + E)
    x = (torch.randn(T, H, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
    wg = (torch.randn(E, H, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    ids, w = ops.moe_router(x, wg, k)
    lg = x.float() @ wg.float().t()
    ri, rw = ref.moe_gate(lg, k)
    top = lg.sort(-1, descending=True).values
    clear = (top[:, k - 1] - top[:, k]) > 1e-3 * lg.abs().amax(-1)  # rows without a near-tie at the cut
    assert clear.sum() > T // 2
    assert torch.equal(ids[clear].long().sort(-1).values, ri[clear].long().sort(-1).values)
    assert torch.allclose(w.sort(-1).values[clear], rw.float().sort(-1).values[clear], atol=1e-4)
    for n in (1, 3, 16):
        i2, w2 = ops.moe_router(x[:n], wg, k)
        assert torch.equal(i2, ids[:n]) and torch.equal(w2, w[:n])


@pytest.mark.parametrize("T", [5, 700, 1500])
def test_moe_ffn_grouped_bitwise_repeatable(T):
    """Routing places pairs in a stable order (no atomic arrival order), so repeated calls on the
    same inputs are bitwise identical, across 1024-pair routing chunks too."""
    H, I, E, k = 256, 128, 8, 2
    g = torch.Generator(device="cuda").manual_seed(T)
    x = (torch.randn(T, H, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
    w13i = (torch.randn(E, 2 * I, H, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    w2 = (torch.randn(E, H, I, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    ids, w = ops.moe_gate(torch.randn(T, E, device="cuda", generator=g), k)
    y0 = ops.moe_ffn_tg(x, ids, w, w13i, w2)
    for _ in range(8):
        assert torch.equal(ops.moe_ffn_tg(x, ids, w, w13i, w2), y0)


def test_moe_ffn_grouped_graph_capture_mixtral_layer():
    """Mixtral-8x7B expert shapes (H 4096, I 14336, E 8, top-2): one captured graph replays decode
    batches with fresh routing and matches the fp32 reference (checked on a row subset)."""
    from distributed_llm_amd.models.llama import gate_up_order
    T, H, I, E, k = 64, 4096, 14336, 8, 2
    g = torch.Generator(device="cuda").manual_seed(3)
    w13 = (torch.randn(E, 2 * I, H, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
    w2 = (torch.randn(E, H, I, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
    w13i = w13.index_select(1, gate_up_order(I).cuda()).contiguous()
    x = torch.zeros(T, H, device="cuda", dtype=torch.bfloat16)
    logits = torch.zeros(T, E, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ids, w = ops.moe_gate(logits, k)
        ops.moe_ffn_tg(x, ids, w, w13i, w2)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        ids, w = ops.moe_gate(logits, k)
        out = ops.moe_ffn_tg(x, ids, w, w13i, w2)
    for _ in range(2):
        x.copy_((torch.randn(T, H, device="cuda", generator=g) * 0.5).to(torch.bfloat16))
        logits.copy_(torch.randn(T, E, device="cuda", generator=g))
        graph.replay()
        torch.cuda.synchronize()
        i2, w2_ = ref.moe_gate(logits, k)
        rows = torch.arange(0, T, 8, device="cuda")
        want = ref.moe_ffn(x[rows], i2[rows], w2_[rows], w13, w2).float()
        err = (out[rows].float() - want).abs().max().item()
        assert err <= 2e-2 * max(1.0, want.abs().max().item()), err


def test_moe_ffn_graph_capture():
    """The MoE path has no host sync: capture once, replay with different routing."""
    T, H, I, E, k = 32, 256, 128, 8, 2
    g = torch.Generator(device="cuda").manual_seed(5)
    w13 = (torch.randn(E, 2 * I, H, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    w2 = (torch.randn(E, H, I, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    x = torch.zeros(T, H, device="cuda", dtype=torch.bfloat16)
    logits = torch.zeros(T, E, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ids, w = ops.moe_gate(logits, k)
        ops.moe_ffn(x, ids, w, w13, w2)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        ids, w = ops.moe_gate(logits, k)
        out = ops.moe_ffn(x, ids, w, w13, w2)
    for it in range(3):
        x.copy_((torch.randn(T, H, device="cuda", generator=g) * 0.5).to(torch.bfloat16))
        logits.copy_(torch.randn(T, E, device="cuda", generator=g))
        graph.replay()
        torch.cuda.synchronize()
        i2, w2_ = ref.moe_gate(logits, k)
        want = ref.moe_ffn(x, i2, w2_, w13, w2).float()
        assert (out.float() - want).abs().max().item() < 2e-2


@pytest.mark.parametrize("H,lo,rows", [(2048, 0, 1000), (4096, 500, 300), (384, 0, 77)])
def test_embedding(H, lo, rows):
    """HIP row gather vs torch indexing; ids outside the vocab shard [lo, lo + rows) give zero rows."""
    torch.manual_seed(0)
    table = bf(rows, H)
    ids = torch.randint(0, lo + rows + 50, (257,), device=DEV, dtype=torch.int32)
    got = ops.embedding(ids, table, lo)
    want = ref.embedding(ids.cpu(), table.cpu(), lo).to(DEV)
    assert torch.equal(got, want)
    ssq = torch.full((300,), float("nan"), device=DEV)      # fused row sums of squares (first layer's scale)
    got2 = ops.embedding(ids, table, lo, ssq_out=ssq)
    assert torch.equal(got2, want)
    torch.testing.assert_close(ssq[:257], (want.float() ** 2).sum(1), rtol=1e-5, atol=1e-4)
    assert torch.isnan(ssq[257:]).all()


@pytest.mark.parametrize("n_ids,ext", [(8, True), (512, True), (64, False)])
def test_step_fetch_and_store(n_ids, ext):
    """Decode-step I/O kernels on device-mapped pinned buffers: dec_dev <- dec_host with the ids
    region taken from d_out where src >= 0; the work list copied as far as its header says; the
    sampled tokens written back to pinned memory."""
    torch.manual_seed(n_ids)
    n_dec, ids_off, src_off = 3 * n_ids + 100, 0, 2 * n_ids + 50
    dec_host = torch.randint(-5, 1000, (n_dec,), dtype=torch.int32).pin_memory()
    src = torch.randint(-1, n_ids, (n_ids,), dtype=torch.int32)
    dec_host[src_off:src_off + n_ids] = src
    d_out = torch.randint(0, 32000, (n_ids + 1,), dtype=torch.int32, device=DEV)
    dec_dev = torch.full((n_dec,), -7, dtype=torch.int32, device=DEV)
    items_host = torch.randint(0, 99, (4 + 4 * 40,), dtype=torch.int32).pin_memory()
    items_host[0] = -13 if ext else 21           # extended list: 4 + 4 * 13 words; plain: 1 + 2 * 21
    items_dev = torch.full((items_host.numel(),), -9, dtype=torch.int32, device=DEV)
    ops.step_fetch(dec_host, dec_dev, ids_off, src_off, n_ids, d_out, items_host, items_dev)
    want = dec_host.clone()
    ids = want[ids_off:ids_off + n_ids]
    m = src >= 0
    ids[m] = d_out.cpu()[src[m].long()]
    torch.cuda.synchronize()
    assert torch.equal(dec_dev.cpu(), want)
    n_it = 4 + 4 * 13 if ext else 1 + 2 * 21
    assert torch.equal(items_dev.cpu()[:n_it], items_host[:n_it])
    assert (items_dev.cpu()[n_it:] == -9).all()
    out_host = torch.zeros(n_ids + 1, dtype=torch.int32).pin_memory()
    ops.step_store(d_out, out_host, n_ids + 1)
    torch.cuda.synchronize()
    assert torch.equal(out_host, d_out.cpu())


@pytest.mark.parametrize("T,n", [(1, 0), (1, 3), (8, 17), (512, 300)])
def test_embedding_with_block_table_scatter(T, n):
    """The decode step's block-table updates ride in the embedding launch (one extra workgroup):
    same rows as the plain gather, same table as ops.scatter_pairs."""
    torch.manual_seed(T + n)
    table = bf(1000, 256)
    ids = torch.randint(0, 1000, (T,), device=DEV, dtype=torch.int32)
    bt = torch.randint(0, 9999, (64, 128), device=DEV, dtype=torch.int32)
    buf = torch.zeros(1 + 2 * 400, dtype=torch.int32, device=DEV)
    idx = torch.randperm(bt.numel(), device=DEV)[:n].to(torch.int32)
    buf[0] = n
    buf[1:1 + 2 * n:2] = idx
    buf[2:2 + 2 * n:2] = torch.arange(n, device=DEV, dtype=torch.int32) + 50000
    want_bt = bt.clone()
    ops.scatter_pairs(want_bt, buf)
    got = ops.embedding(ids, table, 0, scatter=(bt, buf))
    assert torch.equal(got, ref.embedding(ids.cpu(), table.cpu(), 0).to(DEV))
    assert torch.equal(bt, want_bt)


@pytest.mark.parametrize("M", [1, 2, 4, 8])
@pytest.mark.parametrize("N,K,swiglu", [(2560, 2048, False), (2048, 5632, True), (1000, 520, False), (37, 1032, True),
                                         (4096, 3000, True)])
@pytest.mark.parametrize("R", [1, 2, 4])
@pytest.mark.parametrize("grid", [(512, 4, 8192), (8, 64, 0), (1, 0, 0)], ids=["default", "tight", "off"])
def test_gemv(M, N, K, swiglu, R, grid):
    """Small-batch GEMV (csrc/kernels/gemv.hip) vs an fp32 reference; SwiGLU formed on the load;
    N not a multiple of the column block and K not a multiple of 512 exercise the tails."""
    from distributed_llm_amd.ops import gemm as G
    if M * K * 2 > 64 * 1024:
        pytest.skip("X stage exceeds the 64 KB LDS limit (the autotuner never offers it)")
    torch.manual_seed(M * 7 + N)
    x = bf(M, 2 * K if swiglu else K)
    w = bf(N, K, scale=0.05)
    xe = ref.silu_mul(x).float() if swiglu else x.float()
    want = xe @ w.float().t()
    ext = ops._load()
    ext.gemv_set_grid(*grid)   # batch 2-8 grid policy (gemv.hip gemv_grid); restored below
    try:
        got = G._run_plan(("gemv", R), x, w, swiglu, None)
    finally:
        ext.gemv_set_grid(512, 4, 8192)
    torch.testing.assert_close(got.float(), want, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("M", [1, 2, 4, 8])
@pytest.mark.parametrize("N,K", [(2560, 2048), (11264, 2048), (333, 1032)])
def test_gemv_norm(M, N, K):
    """RMSNorm-fused GEMV: y and the new residual match norm kernel semantics (bf16 residual)."""
    if M * K * 2 > 64 * 1024:
        pytest.skip("X stage exceeds the 64 KB LDS limit")
    torch.manual_seed(M + N)
    h, res, nw = bf(M, K), bf(M, K), bf(K)
    w = bf(N, K, scale=0.05)
    res_ref = res.clone()
    xn = ref.rms_norm(h, nw, 1e-5, residual=res_ref)
    want = xn.float() @ w.float().t()
    spare = torch.full_like(res, 7.0)
    y = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    ops._load().gemv_norm(h, res, spare, nw, 1e-5, w, y, 2)
    assert torch.equal(spare, res_ref)
    torch.testing.assert_close(y.float(), want, atol=3e-2, rtol=2e-2)
