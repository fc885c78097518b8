"""Numerics of the fused-epilogue MFMA GEMM (csrc/kernels/tgemm.hip) against plain-PyTorch fp32
references, over every tile / pipeline depth / split-K plan and ragged M, N."""
import math

import pytest
import torch

from distributed_llm_amd import ops
from distributed_llm_amd.ops import gemm as G
from distributed_llm_amd.ops import reference as ref
from distributed_llm_amd.models.llama import fuse_gate_up_weight, fuse_qkv_weight

pytestmark = pytest.mark.gpu

PLANS = [p for p in ([(bm, bn, st, sp, 1, nw) for bm, bn, nw in G._TG_TILES for st in (2, 3) for sp in (1, 3)]
                      + [(bm, bn, 2, sp, 2, nw) for bm, bn, nw in G._TG_TILES for sp in (1, 2)]
                      # deep rings of the 64-row tiles (4 / 6 stages, k-step 64)
                      + [(bm, bn, st, sp, 1, nw) for bm, bn, nw in ((64, 64, 4), (64, 128, 4), (64, 128, 8),
                                                                   (128, 64, 4), (128, 128, 4), (128, 128, 8))
                         for st in (4, 6) for sp in (1, 3)]
                      # two k-groups of 4 waves (KS = 2)
                      + [(bm, bn, st, sp, 2, 4, 2) for bm, bn in ((64, 64), (64, 128), (128, 64), (128, 128))
                         for st in (2, 3) for sp in (1, 2)]
                      # loader-wave plans (NL extra waves stream the ring, the rest only compute)
                      + [(bm, bn, st, sp, 1, nw, 1, nl) for bm, bn, nw, st, nl, _ in G._TG_NL for sp in (1, 3)]
                      # 32-deep k-steps (64-B staged rows): the 256-row tiles with 4-6 stage rings
                      + [(bm, bn, st, sp, 1, 8, 1, nl, 0, 32) for bm, bn, st, nl in G._TG_K32 for sp in (1, 3)]
                      # 32 x 32 x 16 MFMA wave tiles (by_tile_m32), every epilogue, with and without split-K
                      + [p[:3] + (sp,) + p[4:] for p in G._TG_M32 for sp in (1, 3)])
         if p[2] * p[4] * (p[0] + p[1]) * 2 * (p[9] if len(p) > 9 else 64) <= 150 * 1024 and G.tg_built(p)]


def _rnd(*shape, scale=1.0):
    return (torch.randn(*shape, device="cuda") * scale).to(torch.bfloat16)


def _ext():
    return ops._native(torch.empty(1, device="cuda"))


# grid policies of the batch 2-8 GEMV (gemv.hip gemv_grid): the default cap, a cap that leaves
# every workgroup many column blocks, and one workgroup per block (round 5)
GEMV_GRIDS = [(512, 4, 8192), (8, 64, 0), (1, 0, 0)]


@pytest.fixture(params=GEMV_GRIDS, ids=["default", "tight", "off"])
def gemv_grid(request):
    _ext().gemv_set_grid(*request.param)
    yield request.param
    _ext().gemv_set_grid(*GEMV_GRIDS[0])


@pytest.mark.parametrize("plan", PLANS)
@pytest.mark.parametrize("M,N,K", [(1, 64, 256), (37, 200, 384), (130, 320, 1024), (512, 2560, 2048)])
def test_plain(plan, M, N, K):
    torch.manual_seed(M + N + K)
    G.reserve("cuda")
    x, w = _rnd(M, K), _rnd(N, K, scale=0.05)
    y = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    G._tgemm(_ext(), x, w, G.EPI_PLAIN, plan, y=y)
    want = x.float() @ w.float().t()
    torch.testing.assert_close(y.float(), want, atol=2e-2 * want.abs().max().item(), rtol=2e-2)


@pytest.mark.parametrize("plan", PLANS)
def test_plain_row_scale(plan):
    torch.manual_seed(3)
    M, N, K = 70, 128, 512
    G.reserve("cuda")
    x, w = _rnd(M, K), _rnd(N, K, scale=0.05)
    ssq = torch.rand(5, 96, device="cuda") * 10
    y = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    G._tgemm(_ext(), x, w, G.EPI_PLAIN, plan, y=y, ssq_in=ssq, ssq_n=4, norm_scale=1.0 / K, eps=1e-5)
    rinv = torch.rsqrt(ssq[:4, :M].sum(0) / K + 1e-5)
    want = (x.float() @ w.float().t()) * rinv[:, None]
    torch.testing.assert_close(y.float(), want, atol=2e-2 * want.abs().max().item(), rtol=2e-2)


@pytest.mark.parametrize("plan", PLANS)
@pytest.mark.parametrize("M", [5, 200])
def test_residual_add_and_row_sums(plan, M):
    torch.manual_seed(M)
    N, K = 256, 512
    G.reserve("cuda")
    x, w = _rnd(M, K), _rnd(N, K, scale=0.05)
    r = _rnd(M, N)
    r0 = r.clone()
    ssq = torch.full((G.max_slots(N), M), float("nan"), device="cuda")
    G._tgemm(_ext(), x, w, G.EPI_RESADD, plan, y=r, ssq_out=ssq)
    h = (x.float() @ w.float().t()).to(torch.bfloat16)
    want = (h.float() + r0.float()).to(torch.bfloat16)
    torch.testing.assert_close(r.float(), want.float(), atol=3e-2, rtol=2e-2)
    slots = math.ceil(N / plan[1])
    tot = ssq[:slots].sum(0)
    torch.testing.assert_close(tot, (r.float() ** 2).sum(1), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("v_rows", [False, True])
@pytest.mark.parametrize("plan", PLANS)
@pytest.mark.parametrize("d,nq,nkv", [(64, 8, 2), (128, 4, 4), (96, 3, 1)])
def test_qkv_rope_cache(plan, d, nq, nkv, v_rows):
    torch.manual_seed(d)
    M, H = 45, 256
    G.reserve("cuda")
    r = _rnd(M, H)
    ln = (1.0 + 0.1 * torch.randn(H, device="cuda")).to(torch.bfloat16)
    wqkv = _rnd((nq + 2 * nkv) * d, H, scale=0.05)
    wf = fuse_qkv_weight(wqkv, ln, nq, nkv, d)
    ssq = torch.empty(1, M, device="cuda")
    ops.gemm.res_add_ssq(None, r, ssq[0])
    cos_sin = ops.rope_cos_sin(4096, d, 10000.0, "cuda")
    pos = torch.randint(0, 4000, (M,), device="cuda", dtype=torch.int32)
    nblk = 16
    slots = torch.randperm(nblk * 16, device="cuda")[:M].to(torch.int32)
    slots[3] = -1
    kc = torch.zeros(nblk, nkv, 16, d, dtype=torch.bfloat16, device="cuda")
    vc = torch.zeros(nblk, nkv, d, 16, dtype=torch.bfloat16, device="cuda")
    q = torch.empty(M, nq, d, dtype=torch.bfloat16, device="cuda")
    vrow = torch.full((M, nkv * d), float("nan"), dtype=torch.bfloat16, device="cuda") if v_rows else None
    G._tgemm(_ext(), r, wf, G.EPI_QKV, plan, ssq_in=ssq, ssq_n=1, norm_scale=1.0 / H, eps=1e-5, pos=pos,
             cos_sin=cos_sin, slots=slots, q_out=q, kc=kc, vc=vc, nq=nq, nkv=nkv, d=d, v_rows=vrow)
    # reference: rmsnorm -> plain GEMM -> rope + cache write (ops.reference, f32 math)
    x = ref.rms_norm(r.cpu(), ln.cpu(), 1e-5)
    qkv = (x.float() @ wqkv.cpu().float().t()).to(torch.bfloat16)
    kr = torch.zeros(nblk, nkv, 16, d, dtype=torch.bfloat16)
    vr = torch.zeros(nblk, nkv, d, 16, dtype=torch.bfloat16)
    qr = ref.rope_and_cache(qkv, pos.cpu(), cos_sin.cpu(), slots.cpu(), kr, vr, nq, nkv, d)
    torch.testing.assert_close(q.cpu().float(), qr.float(), atol=4e-2, rtol=3e-2)
    torch.testing.assert_close(kc.cpu().float(), kr.float(), atol=4e-2, rtol=3e-2)
    if v_rows:
        # V handed over row-major (every row, slot or not); the V^T cache is left to the attention kernel
        v_ref = qkv[:, (nq + nkv) * d:].float()
        torch.testing.assert_close(vrow.cpu().float(), v_ref, atol=4e-2, rtol=3e-2)
        assert (vc == 0).all()
    else:
        torch.testing.assert_close(vc.cpu().float(), vr.float(), atol=4e-2, rtol=3e-2)


@pytest.mark.parametrize("plan", PLANS)
def test_swiglu(plan):
    torch.manual_seed(7)
    M, H, I = 99, 256, 320
    G.reserve("cuda")
    r = _rnd(M, H)
    ln = (1.0 + 0.1 * torch.randn(H, device="cuda")).to(torch.bfloat16)
    wgu = _rnd(2 * I, H, scale=0.05)
    wf = fuse_gate_up_weight(wgu, ln)
    ssq = torch.empty(1, M, device="cuda")
    ops.gemm.res_add_ssq(None, r, ssq[0])
    act = torch.empty(M, I, dtype=torch.bfloat16, device="cuda")
    G._tgemm(_ext(), r, wf, G.EPI_SWIGLU, plan, y=act, ssq_in=ssq, ssq_n=1, norm_scale=1.0 / H, eps=1e-5)
    x = ref.rms_norm(r.cpu(), ln.cpu(), 1e-5)
    gu = (x.float() @ wgu.cpu().float().t()).to(torch.bfloat16)
    want = ref.silu_mul(gu)
    torch.testing.assert_close(act.cpu().float(), want.float(), atol=3e-2, rtol=3e-2)


def test_res_add_ssq():
    torch.manual_seed(1)
    h, r = _rnd(33, 320), _rnd(33, 320)
    r0 = r.clone()
    ssq = torch.empty(33, device="cuda")
    ops.gemm.res_add_ssq(h, r, ssq)
    want = (h.float() + r0.float()).to(torch.bfloat16)
    assert torch.equal(r, want)
    torch.testing.assert_close(ssq, (want.float() ** 2).sum(1), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("H,slots", [(2048, 8), (2048, 3), (320, 5), (4096, 64)])
def test_res_add_ssq_sliced(H, slots):
    """Partial sums over column slices ([slots, M] form): the slices cover H exactly once."""
    torch.manual_seed(H + slots)
    h, r = _rnd(37, H), _rnd(37, H)
    r0 = r.clone()
    ssq = torch.full((slots, 40), float("nan"), device="cuda")
    n = ops.gemm.res_add_ssq(h, r, ssq)
    cw = math.ceil(math.ceil(H / slots) / 512) * 512   # whole 512-column wave passes per slice
    assert n == math.ceil(H / cw) and 1 <= n <= slots
    want = (h.float() + r0.float()).to(torch.bfloat16)
    assert torch.equal(r, want)
    torch.testing.assert_close(ssq[:n, :37].sum(0), (want.float() ** 2).sum(1), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("core,M", [("tg", 77), ("blas", 77), ("gemv1", 1), ("gemv2", 8), ("gemv4", 4), ("gemv1", 2)])
def test_fused_ops_both_cores(core, M, monkeypatch):
    """The fused decoder ops give the same results through the tgemm epilogue, through the
    vendor GEMM + standalone epilogue kernels (qkv_post / res_add_ssq / swiglu_post) and, at
    batch <= 8, through the fused-epilogue GEMV (gemv.hip EPI)."""
    monkeypatch.setenv("DLLM_FUSED_CORE", core)
    torch.manual_seed(11)
    H, I, d, nq, nkv = 256, 384, 64, 4, 2
    G.reserve("cuda")
    r = _rnd(M, H)
    if core.startswith("gemv"):
        assert G.fused_gemv_r(r, (nq + 2 * nkv) * d) == int(core[4:])   # the GEMV path really runs
    ln1 = (1.0 + 0.1 * torch.randn(H, device="cuda")).to(torch.bfloat16)
    ln2 = (1.0 + 0.1 * torch.randn(H, device="cuda")).to(torch.bfloat16)
    wqkv, wo = _rnd((nq + 2 * nkv) * d, H, scale=0.05), _rnd(H, nq * d, scale=0.05)
    wgu, wd = _rnd(2 * I, H, scale=0.05), _rnd(H, I, scale=0.05)
    ssq = torch.empty(G.max_slots(H, M), M, device="cuda")
    ops.gemm.res_add_ssq(None, r, ssq[0])
    cos_sin = ops.rope_cos_sin(512, d, 10000.0, "cuda")
    pos = torch.arange(M, device="cuda", dtype=torch.int32)
    slots = torch.arange(M, device="cuda", dtype=torch.int32)
    kc = torch.zeros(8, nkv, 16, d, dtype=torch.bfloat16, device="cuda")
    vc = torch.zeros(8, nkv, d, 16, dtype=torch.bfloat16, device="cuda")
    r_ref = r.cpu().clone()
    q = G.qkv_rope_cache(r, fuse_qkv_weight(wqkv, ln1, nq, nkv, d), ssq, 1, 1e-5, pos, cos_sin, slots, kc, vc,
                         nq, nkv, d)
    o = _rnd(M, nq * d)
    ssq2 = torch.empty(G.max_slots(H, M), M, device="cuda")
    n2 = G.matmul_resadd(o, wo, r, ssq2)
    act = G.swiglu_matmul(r, fuse_gate_up_weight(wgu, ln2), ssq2, n2, 1e-5)
    r_after_wo = r.cpu().clone()
    ssq3 = torch.full((G.max_slots(H, M), M), float("nan"), device="cuda")
    n3 = G.matmul_resadd(act, wd, r, ssq3)
    # fp32 references
    x = ref.rms_norm(r_ref, ln1.cpu(), 1e-5)
    qkv = (x.float() @ wqkv.cpu().float().t()).to(torch.bfloat16)
    kr = torch.zeros(8, nkv, 16, d, dtype=torch.bfloat16)
    vr = torch.zeros(8, nkv, d, 16, dtype=torch.bfloat16)
    qr = ref.rope_and_cache(qkv, pos.cpu(), cos_sin.cpu(), slots.cpu(), kr, vr, nq, nkv, d)
    h = (o.cpu().float() @ wo.cpu().float().t()).to(torch.bfloat16)
    r2 = (h.float() + r_ref.float()).to(torch.bfloat16)
    x2 = ref.rms_norm(r2, ln2.cpu(), 1e-5)
    ar = ref.silu_mul((x2.float() @ wgu.cpu().float().t()).to(torch.bfloat16))
    torch.testing.assert_close(q.cpu().float(), qr.float(), atol=4e-2, rtol=3e-2)
    torch.testing.assert_close(kc.cpu().float(), kr.float(), atol=4e-2, rtol=3e-2)
    torch.testing.assert_close(vc.cpu().float(), vr.float(), atol=4e-2, rtol=3e-2)
    torch.testing.assert_close(r_after_wo.float(), r2.float(), atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(act.cpu().float(), ar.float(), atol=3e-2, rtol=3e-2)
    # down projection: residual add and the row sums of squares its slots hold
    r3 = ((act.cpu().float() @ wd.cpu().float().t()).to(torch.bfloat16).float() + r_after_wo.float()).to(torch.bfloat16)
    torch.testing.assert_close(r.cpu().float(), r3.float(), atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(ssq3[:n3].sum(0).cpu(), (r.cpu().float() ** 2).sum(1), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("M", [5, 77, 512])
@pytest.mark.parametrize("nq,nkv,d", [(4, 2, 64), (32, 4, 64), (8, 2, 128)])
def test_qkv_post_v_rows(M, nq, nkv, d, monkeypatch):
    """Vendor core + standalone QKV epilogue (qkv_post) in the decode hand-over form: q and K as
    the reference, V row-major into v_new (what the attention kernel moves into V^T), the V^T
    cache untouched; without v_new, V^T written as before."""
    monkeypatch.setenv("DLLM_FUSED_CORE", "blas")
    torch.manual_seed(M + nq + d)
    H = 256
    G.reserve("cuda")
    r = _rnd(M, H)
    ln1 = (1.0 + 0.1 * torch.randn(H, device="cuda")).to(torch.bfloat16)
    wqkv = _rnd((nq + 2 * nkv) * d, H, scale=0.05)
    ssq = torch.empty(G.max_slots(H, M), M, device="cuda")
    ops.gemm.res_add_ssq(None, r, ssq[0])
    cos_sin = ops.rope_cos_sin(1024, d, 10000.0, "cuda")
    pos = torch.randint(0, 1000, (M,), device="cuda", dtype=torch.int32)
    nb = (M + 15) // 16 + 4
    slots = torch.randperm(nb * 16, device="cuda")[:M].to(torch.int32)
    wf = fuse_qkv_weight(wqkv, ln1, nq, nkv, d)
    x = ref.rms_norm(r.cpu(), ln1.cpu(), 1e-5)
    qkv = (x.float() @ wqkv.cpu().float().t()).to(torch.bfloat16)
    kr = torch.zeros(nb, nkv, 16, d, dtype=torch.bfloat16)
    vr = torch.zeros(nb, nkv, d, 16, dtype=torch.bfloat16)
    qr = ref.rope_and_cache(qkv, pos.cpu(), cos_sin.cpu(), slots.cpu(), kr, vr, nq, nkv, d)
    s_cpu = slots.cpu().long()
    v_rows_ref = vr[s_cpu // 16, :, :, s_cpu % 16].reshape(M, nkv * d)
    for with_v in (True, False):
        kc = torch.zeros(nb, nkv, 16, d, dtype=torch.bfloat16, device="cuda")
        vc = torch.zeros(nb, nkv, d, 16, dtype=torch.bfloat16, device="cuda")
        vn = torch.full((M, nkv * d), float("nan"), dtype=torch.bfloat16, device="cuda") if with_v else None
        out = G.qkv_rope_cache(r, wf, ssq, 1, 1e-5, pos, cos_sin, slots, kc, vc, nq, nkv, d, v_new=vn)
        q, used = out if with_v else (out, None)
        torch.testing.assert_close(q.cpu().float(), qr.float(), atol=4e-2, rtol=3e-2)
        torch.testing.assert_close(kc.cpu().float(), kr.float(), atol=4e-2, rtol=3e-2)
        if with_v:
            assert used is vn
            torch.testing.assert_close(vn.cpu().float(), v_rows_ref.float(), atol=4e-2, rtol=3e-2)
            assert not vc.any()
        else:
            torch.testing.assert_close(vc.cpu().float(), vr.float(), atol=4e-2, rtol=3e-2)


@pytest.mark.parametrize("M", [1, 2, 4, 8])
@pytest.mark.parametrize("R", [1, 2, 4])
@pytest.mark.parametrize("N,K", [(256, 512), (2048, 2048), (4096, 5632), (2048, 5632), (1024, 3000), (1024, 14336)])
# (2048, 5632) / (1024, 3000) at M <= 2, R = 1: the whole-row 12- / 8-load trips (gemv.hip launch_gemv)
def test_gemv_resadd(M, R, N, K, gemv_grid):
    """Fused-epilogue GEMV, residual form: r += bf16(x . w^T), one partial row sum per workgroup."""
    if M * K * 2 > 64 * 1024:
        pytest.skip("X does not fit the GEMV's 64 KB LDS stage")
    torch.manual_seed(M * 7 + R + N)
    x, w, r = _rnd(M, K), _rnd(N, K, scale=0.05), _rnd(M, N)
    r0 = r.clone()
    ssq = torch.full((G.max_slots(N, M), M), float("nan"), device="cuda")
    n = _ext().gemv_resadd(x, w, r, ssq, R)
    assert n == _ext().gemv_slots(M, N, R) and 1 <= n <= math.ceil(N / (4 * R))
    if gemv_grid[1] == 0 or M == 1:
        assert n == math.ceil(N / (4 * R))
    want = ((x.float() @ w.float().t()).to(torch.bfloat16).float() + r0.float()).to(torch.bfloat16)
    torch.testing.assert_close(r.float(), want.float(), atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(ssq[:n].sum(0), (r.float() ** 2).sum(1), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("M", [1, 2, 4, 8])
@pytest.mark.parametrize("R", [1, 2, 4])
@pytest.mark.parametrize("d,nq,nkv,H", [(64, 8, 2, 256), (128, 32, 8, 4096), (96, 3, 1, 512), (64, 32, 4, 2048)])
def test_gemv_qkv(M, R, d, nq, nkv, H, gemv_grid):
    """Fused-epilogue GEMV, QKV form (paired columns): folded RMSNorm row scale from partial sums,
    RoPE, q out, K and V^T into the paged caches; vs rmsnorm -> fp32 GEMM -> rope + cache write."""
    if M * H * 2 > 64 * 1024:
        pytest.skip("X does not fit the GEMV's 64 KB LDS stage")
    torch.manual_seed(M + R + d)
    r = _rnd(M, H)
    ln = (1.0 + 0.1 * torch.randn(H, device="cuda")).to(torch.bfloat16)
    wqkv = _rnd((nq + 2 * nkv) * d, H, scale=0.05)
    wf = fuse_qkv_weight(wqkv, ln, nq, nkv, d)
    ssq = torch.empty(G.max_slots(H, M), M, device="cuda")
    n = ops.gemm.res_add_ssq(None, r, ssq)
    cos_sin = ops.rope_cos_sin(4096, d, 10000.0, "cuda")
    pos = torch.randint(0, 4000, (M,), device="cuda", dtype=torch.int32)
    nblk = 4
    slots = torch.randperm(nblk * 16, device="cuda")[:M].to(torch.int32)
    if M > 2:
        slots[1] = -1
    kc = torch.zeros(nblk, nkv, 16, d, dtype=torch.bfloat16, device="cuda")
    vc = torch.zeros(nblk, nkv, d, 16, dtype=torch.bfloat16, device="cuda")
    q = torch.empty(M, nq, d, dtype=torch.bfloat16, device="cuda")
    _ext().gemv_qkv(r, wf, ssq, n, 1.0 / H, 1e-5, pos, cos_sin, slots, q, kc, vc, nq, nkv, d, R)
    x = ref.rms_norm(r.cpu(), ln.cpu(), 1e-5)
    qkv = (x.float() @ wqkv.cpu().float().t()).to(torch.bfloat16)
    kr = torch.zeros(nblk, nkv, 16, d, dtype=torch.bfloat16)
    vr = torch.zeros(nblk, nkv, d, 16, dtype=torch.bfloat16)
    qr = ref.rope_and_cache(qkv, pos.cpu(), cos_sin.cpu(), slots.cpu(), kr, vr, nq, nkv, d)
    # gamma folded into bf16 weights + the row scale applied after the K-sum: rounding differs from
    # the normalise-then-multiply reference by up to ~1 bf16 ulp of the largest outputs
    tol = max(4e-2, 8e-3 * qr.float().abs().max().item())
    torch.testing.assert_close(q.cpu().float(), qr.float(), atol=tol, rtol=3e-2)
    torch.testing.assert_close(kc.cpu().float(), kr.float(), atol=tol, rtol=3e-2)
    torch.testing.assert_close(vc.cpu().float(), vr.float(), atol=tol, rtol=3e-2)


@pytest.mark.parametrize("M", [1, 2, 4, 8])
@pytest.mark.parametrize("R", [1, 2, 4])
@pytest.mark.parametrize("H,I", [(256, 320), (2048, 5632)])
def test_gemv_swiglu(M, R, H, I, gemv_grid):
    """Fused-epilogue GEMV, SwiGLU form: act = silu(g) * u of the folded-norm gate|up product."""
    torch.manual_seed(M + R + I)
    r = _rnd(M, H)
    ln = (1.0 + 0.1 * torch.randn(H, device="cuda")).to(torch.bfloat16)
    wgu = _rnd(2 * I, H, scale=0.05)
    wf = fuse_gate_up_weight(wgu, ln)
    ssq = torch.empty(G.max_slots(H, M), M, device="cuda")
    n = ops.gemm.res_add_ssq(None, r, ssq)
    act = torch.empty(M, I, dtype=torch.bfloat16, device="cuda")
    _ext().gemv_swiglu(r, wf, ssq, n, 1.0 / H, 1e-5, act, R)
    x = ref.rms_norm(r.cpu(), ln.cpu(), 1e-5)
    want = ref.silu_mul((x.float() @ wgu.cpu().float().t()).to(torch.bfloat16))
    tol = max(3e-2, 8e-3 * want.abs().max().item())   # about 1 bf16 ulp of the largest output (test_gemv_qkv)
    torch.testing.assert_close(act.cpu().float(), want.float(), atol=tol, rtol=3e-2)


@pytest.mark.parametrize("M", [1, 2, 8])
@pytest.mark.parametrize("R", [1, 2])
def test_gemv_swiglu_partials_past_1024_slots(M, R):
    """The PAIRED GEMV requests its first row's first 1024 partial sums ahead of the weight stream
    and sums any further slots (and rows past the fourth) afterwards: the same partials spread over
    1,500 slots, half in the first 1,024 and half after, give the same activation."""
    H, I = 512, 640
    torch.manual_seed(M + 31 * R)
    r = _rnd(M, H)
    ln = (1.0 + 0.1 * torch.randn(H, device="cuda")).to(torch.bfloat16)
    wgu = _rnd(2 * I, H, scale=0.05)
    wf = fuse_gate_up_weight(wgu, ln)
    ssq = torch.empty(G.max_slots(H, M), M, device="cuda")
    n = ops.gemm.res_add_ssq(None, r, ssq)
    big = torch.zeros(1500, M, device="cuda")
    big[:n] = ssq[:n] / 2
    big[1100:1100 + n] = ssq[:n] / 2
    act_ref = torch.empty(M, I, dtype=torch.bfloat16, device="cuda")
    act = torch.empty(M, I, dtype=torch.bfloat16, device="cuda")
    _ext().gemv_swiglu(r, wf, ssq, n, 1.0 / H, 1e-5, act_ref, R)
    _ext().gemv_swiglu(r, wf, big, 1500, 1.0 / H, 1e-5, act, R)
    torch.testing.assert_close(act.float(), act_ref.float(), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("plan", PLANS)
@pytest.mark.parametrize("M,N,K", [(37, 200, 384), (320, 2048, 2048)])
def test_panel_weight_matches_row_major(plan, M, N, K):
    """The K-panel-major weight copy (GemmArgs.w_panel) streams the same tiles in the same k order:
    bit-identical outputs to the row-major weight for every plan, split-K included."""
    torch.manual_seed(M * 7 + N)
    G.reserve("cuda")
    x, w = _rnd(M, K), _rnd(N, K, scale=0.05)
    wp = G.panel_weight(w)
    assert G._nk(wp) == (N, K)
    a = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    b = torch.empty_like(a)
    G._tgemm(_ext(), x, w, G.EPI_PLAIN, plan, y=a)
    G._tgemm(_ext(), x, wp, G.EPI_PLAIN, plan, y=b)
    assert torch.equal(a, b)


@pytest.mark.parametrize("M", [5, 200])
def test_panel_weight_fused_epilogues(M):
    """RESADD / SWIGLU / QKV through the fused ops with the panel copy (wp=) equal the row-major run."""
    torch.manual_seed(21 + M)
    G.reserve("cuda")
    H, I, nq, nkv, d = 512, 768, 8, 2, 64
    plan = G.tg_plan(M, 2 * I, H)
    r0 = _rnd(M, H)
    w_gu, w_o = _rnd(2 * I, H, scale=0.05), _rnd(H, I, scale=0.05)
    ssq = torch.rand(3, M, device="cuda") * 10 + 1
    outs = []
    for panel in (False, True):
        act = G.swiglu_matmul(r0, w_gu, ssq, 3, 1e-5, wp=G.panel_weight(w_gu) if panel else None)
        r = r0.clone()
        so = torch.zeros(64, M, device="cuda")
        n = G.matmul_resadd(act, w_o, r, so, wp=G.panel_weight(w_o) if panel else None)
        outs.append((act, r, so[:n]))
    for u, v in zip(*outs):
        assert torch.equal(u, v)
    assert plan


SK_PLANS = sorted((bm, bn, st, 1, ks, nw, 1, nl, 1) for bm, bn, st, ks, nw, nl in G._SK_PLANS)


@pytest.mark.parametrize("plan", SK_PLANS)
@pytest.mark.parametrize("M,N,K", [(320, 2048, 2048), (37, 200, 384), (130, 320, 1024), (300, 2560, 5632)])
def test_stream_k_plain(plan, M, N, K):
    """Stream-K (one workgroup per CU walking equal shares of tiles x k-steps, tiles split over
    workgroups combined by their last arriver) against the fp32 reference; deterministic sums."""
    torch.manual_seed(M + 3 * N + K)
    G.reserve("cuda")
    x, w = _rnd(M, K), _rnd(N, K, scale=0.05)
    y = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    G._tgemm(_ext(), x, w, G.EPI_PLAIN, plan, y=y)
    want = x.float() @ w.float().t()
    torch.testing.assert_close(y.float(), want, atol=2e-2 * want.abs().max().item(), rtol=2e-2)
    y2 = torch.empty_like(y)
    G._tgemm(_ext(), x, G.panel_weight(w), G.EPI_PLAIN, plan, y=y2)   # tickets re-armed, panel weights
    assert torch.equal(y, y2)


def test_stream_k_fused_and_pruned_plans_refused():
    """Stream-K plans are built for the PLAIN epilogue only, and the pruned plans (tgemm.hip kPruned)
    not at all: both are refused with an error, never launched."""
    G.reserve("cuda")
    x, w = _rnd(320, 512), _rnd(1024, 512, scale=0.05)
    y = torch.empty(320, 1024, dtype=torch.bfloat16, device="cuda")
    with pytest.raises(ValueError):
        G._tgemm(_ext(), x, w, G.EPI_RESADD, SK_PLANS[0], y=y, ssq_out=torch.zeros(64, 320, device="cuda"))
    for key in sorted(G._TG_PRUNED):
        bm, bn, st, ks, nw, wk, nl, bk, mf = key
        plan = (bm, bn, st, 1, ks, nw, wk, nl, 0, bk, mf)
        assert not G.tg_built(plan)
        with pytest.raises(RuntimeError):
            G._tgemm(_ext(), x, w, G.EPI_PLAIN, plan, y=y)


# ---- small-batch MFMA GEMM with the fused epilogues (skinny_gemm.hip skinny_epi_kernel, M <= 16)
SKE_SPLITS = [1, 3]


@pytest.mark.parametrize("M", [1, 3, 8, 16])
@pytest.mark.parametrize("panel", [False, True])
@pytest.mark.parametrize("sp", SKE_SPLITS)
@pytest.mark.parametrize("N,K", [(256, 512), (2048, 2048), (2048, 5632), (96, 320)])
def test_skinny_epi_plain_and_resadd(M, panel, sp, N, K):
    if K % 64:
        pytest.skip("panel / skE weights need K % 64 == 0")
    torch.manual_seed(M * 7 + N + sp)
    G.reserve("cuda")
    x, w, r = _rnd(M, K), _rnd(N, K, scale=0.05), _rnd(M, N)
    wl = G.panel_weight(w) if panel else w
    y = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    G.skinny_epi(x, wl, G.EPI_PLAIN, sp, y=y)
    want = x.float() @ w.float().t()
    torch.testing.assert_close(y.float(), want, atol=2e-2 * want.abs().max().item(), rtol=2e-2)
    r0 = r.clone()
    ssq = torch.full((G.max_slots(N, M), M), float("nan"), device="cuda")
    n = G.skinny_epi(x, wl, G.EPI_RESADD, sp, res=r, ssq_out=ssq)
    assert n == math.ceil(N / 32)
    want = (want.to(torch.bfloat16).float() + r0.float()).to(torch.bfloat16)
    torch.testing.assert_close(r.float(), want.float(), atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(ssq[:n].sum(0), (r.float() ** 2).sum(1), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("M", [1, 4, 8, 16])
@pytest.mark.parametrize("panel", [False, True])
@pytest.mark.parametrize("sp", SKE_SPLITS)
@pytest.mark.parametrize("d,nq,nkv,H", [(64, 8, 2, 256), (128, 32, 8, 4096), (64, 32, 4, 2048)])
def test_skinny_epi_qkv(M, panel, sp, d, nq, nkv, H):
    """QKV form: folded RMSNorm row scale, RoPE on the permuted (c, c + 16) pairs, q out, K and V^T
    into the paged caches; vs rmsnorm -> fp32 GEMM -> rope + cache write (as test_gemv_qkv)."""
    torch.manual_seed(M + d + sp)
    G.reserve("cuda")
    r = _rnd(M, H)
    ln = (1.0 + 0.1 * torch.randn(H, device="cuda")).to(torch.bfloat16)
    wqkv = _rnd((nq + 2 * nkv) * d, H, scale=0.05)
    wf = fuse_qkv_weight(wqkv, ln, nq, nkv, d)
    ssq = torch.empty(G.max_slots(H, M), M, device="cuda")
    n = ops.gemm.res_add_ssq(None, r, ssq)
    cos_sin = ops.rope_cos_sin(4096, d, 10000.0, "cuda")
    pos = torch.randint(0, 4000, (M,), device="cuda", dtype=torch.int32)
    nblk = 4
    slots = torch.randperm(nblk * 16, device="cuda")[:M].to(torch.int32)
    if M > 2:
        slots[1] = -1
    kc = torch.zeros(nblk, nkv, 16, d, dtype=torch.bfloat16, device="cuda")
    vc = torch.zeros(nblk, nkv, d, 16, dtype=torch.bfloat16, device="cuda")
    q = torch.empty(M, nq, d, dtype=torch.bfloat16, device="cuda")
    G.skinny_epi(r, G.panel_weight(wf) if panel else wf, G.EPI_QKV, sp, ssq_in=ssq, ssq_n=n, scale=1.0 / H, eps=1e-5,
                 pos=pos, cos_sin=cos_sin, slots=slots, q_out=q, kc=kc, vc=vc, nq=nq, nkv=nkv, d=d)
    x = ref.rms_norm(r.cpu(), ln.cpu(), 1e-5)
    qkv = (x.float() @ wqkv.cpu().float().t()).to(torch.bfloat16)
    kr = torch.zeros(nblk, nkv, 16, d, dtype=torch.bfloat16)
    vr = torch.zeros(nblk, nkv, d, 16, dtype=torch.bfloat16)
    qr = ref.rope_and_cache(qkv, pos.cpu(), cos_sin.cpu(), slots.cpu(), kr, vr, nq, nkv, d)
    tol = max(4e-2, 8e-3 * qr.float().abs().max().item())
    torch.testing.assert_close(q.cpu().float(), qr.float(), atol=tol, rtol=3e-2)
    torch.testing.assert_close(kc.cpu().float(), kr.float(), atol=tol, rtol=3e-2)
    torch.testing.assert_close(vc.cpu().float(), vr.float(), atol=tol, rtol=3e-2)


@pytest.mark.parametrize("M", [1, 5, 8, 16])
@pytest.mark.parametrize("panel", [False, True])
@pytest.mark.parametrize("sp", SKE_SPLITS)
@pytest.mark.parametrize("H,I", [(256, 320), (2048, 5632)])
def test_skinny_epi_swiglu(M, panel, sp, H, I):
    torch.manual_seed(M + I + sp)
    G.reserve("cuda")
    r = _rnd(M, H)
    ln = (1.0 + 0.1 * torch.randn(H, device="cuda")).to(torch.bfloat16)
    wgu = _rnd(2 * I, H, scale=0.05)
    wf = fuse_gate_up_weight(wgu, ln)
    ssq = torch.empty(G.max_slots(H, M), M, device="cuda")
    n = ops.gemm.res_add_ssq(None, r, ssq)
    act = torch.empty(M, I, dtype=torch.bfloat16, device="cuda")
    G.skinny_epi(r, G.panel_weight(wf) if panel else wf, G.EPI_SWIGLU, sp, y=act, ssq_in=ssq, ssq_n=n, scale=1.0 / H,
                 eps=1e-5)
    x = ref.rms_norm(r.cpu(), ln.cpu(), 1e-5)
    want = ref.silu_mul((x.float() @ wgu.cpu().float().t()).to(torch.bfloat16))
    tol = max(3e-2, 8e-3 * want.abs().max().item())
    torch.testing.assert_close(act.cpu().float(), want.float(), atol=tol, rtol=3e-2)


@pytest.mark.parametrize("M", [4, 64])
def test_fused_core_timed_in_situ(M):
    """The autotuner times every fused-op core option of a decoder layer through the fused op
    itself (ops.gemm._retime_fused): each option runs, and the chosen core is the fastest of them."""
    G.reserve("cuda")
    H, I, nq, nkv, d = 512, 1024, 8, 2, 64
    fused = [((nq + 2 * nkv) * d, H), (H, nq * d), (2 * I, H), (H, I)]
    shapes = sorted({(n, k, False) for n, k in fused})
    saved = (dict(G._P.fused_core), dict(G._P.fused_opts), dict(G._P.tg_plans), dict(G._P.plans))
    try:
        G.autotune(shapes, [M], "cuda", fused=fused, qkv_dims=(nq, nkv, d))
        for n, k in fused:
            opts = G._P.fused_opts[(M, n, k)]
            assert opts and all(math.isfinite(t) and t > 0 for t in opts.values()), opts
            core, best = G._P.fused_core[(M, n, k)], min(opts, key=opts.get)
            # the fastest option, or a one-launch core within SPLIT_MARGIN of a faster split form
            assert core == best or (best == "lin" and core != "lin" and opts[core] <= G.SPLIT_MARGIN * opts["lin"]
                                    and opts[core] == min(t for c, t in opts.items() if c != "lin"))
    finally:
        for dst, src in zip((G._P.fused_core, G._P.fused_opts, G._P.tg_plans, G._P.plans), saved):
            dst.clear()
            dst.update(src)
