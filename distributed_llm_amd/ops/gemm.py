"""Linear layers on hand-written MFMA kernels, autotuned per decode bucket, with fused epilogues.

``linear(x, w)`` computes ``x @ w.T`` (w stored [N, K], K contiguous).
``linear_swiglu(gu, w)`` computes ``silu(gu[:, :K]) * gu[:, K:] @ w.T``.

Kernels (csrc/kernels):
  * ``tgemm.hip``  — LDS-tiled MFMA GEMM (global_load_lds ring, XOR-swizzled LDS, XCD-aware
    block order, optional in-launch split-K) with the transformer epilogues used by the fused
    decoder layer (models/llama.py): QKV + RoPE + paged-KV write, residual add + row sums of
    squares (RMSNorm folded into the next GEMM), SwiGLU.  Any M (decode buckets and prefill).
  * ``gemv.hip`` (M <= 8), ``skinny_gemm.hip`` (M <= 128): register-streaming decode GEMMs without
    LDS tiling.
  * hipBLASLt via ``F.linear`` stays a candidate, so a custom kernel is used only where it wins.

Plans are measured once per (M, N, K) OUTSIDE graph capture (``autotune``, called by the engine
for every decode bucket before capturing) as hipGraph replays over rotated weight copies (a
decode step streams the whole model: weights come from HBM, not the Infinity Cache); an unseen
shape (prefill) uses a heuristic plan.  CPU tensors -> plain torch.

Split-K workspaces are FIXED-size per (device, owner) and never re-allocated: captured graphs
keep raw pointers to them, so growing (freeing) a workspace after a capture would leave graph
replays writing into freed memory.  Plans whose workspace need exceeds the fixed
size are never chosen.  Engines capture under their own owner key (``workspace_owner``), so two
engines replaying graphs concurrently on one device never share split-K tickets.
"""
from __future__ import annotations

import contextlib
import contextvars
import math
import os
from typing import Dict, Iterable, Optional, Tuple

import torch
import torch.nn.functional as F

from . import _native, reference as ref

MAX_M = 1024       # decode buckets up to this size are autotuned
SKINNY_MAX_M = 128
_SPLITS = (1, 2, 4, 8, 16)
_NTWS = (1, 2, 4)
_GEMV_MS = (1, 2, 4, 8)   # csrc/kernels/gemv.hip instantiations (decode buckets below 16)
SKE_MAX_M = 16            # small-batch MFMA GEMM with fused epilogues (skinny_gemm.hip skinny_epi_kernel)
_SKE_SPLITS = (1, 2, 4, 8)
_GEMV_RS = (1, 2, 4)
_TG_TILES = ((64, 64, 4), (64, 128, 4), (128, 64, 4), (128, 128, 4), (64, 128, 8), (128, 128, 8), (192, 128, 8),
             (256, 128, 8),
             (256, 256, 8))
_TG_SPLITS = (1, 2, 3, 4, 6, 8)
# loader-wave plans (csrc/kernels/tgemm.hip by_tile_nl): (bm, bn, compute waves, stages, loader waves);
# M is the smallest batch each is tried at (larger tiles only pay once M fills them)
# (8 loader waves: a CU's LDS-DMA intake grows with the waves issuing it, ~75 GB/s at 4 and ~140 GB/s
# at 8 on contiguous pieces, scripts/exp/intake.hip; profiles/r3_decode_gemm_panel.md)
_TG_NL = ((16, 128, 4, 4, 6, 1), (16, 128, 4, 8, 6, 1),   # batch <= 16 only (TG_NL16_MAX_M): 16-row tiles
          (64, 64, 4, 4, 4, 1), (128, 64, 4, 4, 4, 65), (160, 128, 8, 3, 4, 129), (256, 128, 8, 3, 4, 129),
          (64, 64, 4, 4, 8, 1), (64, 64, 4, 8, 8, 1), (128, 64, 4, 4, 8, 65), (128, 128, 4, 4, 8, 65),
          (160, 128, 8, 3, 6, 129), (256, 128, 8, 3, 8, 129))
# 32-deep k-step plans (csrc/kernels/tgemm.hip by_tile_k32): (bm, bn, stages, loaders), 8 compute waves;
# as plan tuples (bm, bn, stages, splits, 1, 8, 1, loaders, 0, 32)
_TG_K32 = ((256, 256, 4, 0),)
# 32 x 32 x 16 MFMA plans (csrc/kernels/tgemm.hip by_tile_m32), as full plan tuples with k depth 64 and
# mfma 32: the flagship's 64-row decode tiles, measured against everything else (the 128- and 256-row
# forms lost 6-16 % to 16 x 16 x 32 and are pruned: profiles/r6_gemm_fill_path.md, r6_prune.md)
_TG_M32 = ((64, 64, 3, 1, 2, 4, 1, 0, 0, 64, 32), (64, 128, 3, 1, 2, 8, 1, 0, 0, 64, 32))
# plans no measured shape ever selected, not instantiated (csrc/kernels/tgemm.hip kPruned, same table):
# (bm, bn, stages, ks, waves, wk, loaders, k depth, mfma); profiles/r6_prune.md
_TG_PRUNED = frozenset({
    (64, 128, 6, 1, 4, 1, 0, 64, 16), (64, 128, 2, 2, 4, 1, 0, 64, 16), (128, 64, 3, 1, 4, 1, 0, 64, 16),
    (128, 64, 4, 1, 4, 1, 0, 64, 16), (128, 64, 6, 1, 4, 1, 0, 64, 16), (128, 64, 2, 2, 4, 1, 0, 64, 16),
    (128, 64, 3, 2, 4, 1, 0, 64, 16), (128, 128, 3, 1, 4, 1, 0, 64, 16), (128, 128, 4, 1, 4, 1, 0, 64, 16),
    (128, 128, 2, 2, 4, 1, 0, 64, 16), (64, 128, 2, 1, 8, 1, 0, 64, 16), (64, 128, 2, 2, 8, 1, 0, 64, 16),
    (128, 128, 2, 1, 8, 1, 0, 64, 16), (128, 128, 2, 2, 8, 1, 0, 64, 16), (192, 128, 2, 1, 8, 1, 0, 64, 16),
    (256, 128, 2, 1, 8, 1, 0, 64, 16), (64, 128, 2, 2, 4, 2, 0, 64, 16),
    (128, 64, 2, 2, 4, 2, 0, 64, 16), (128, 64, 3, 2, 4, 2, 0, 64, 16), (128, 128, 2, 2, 4, 2, 0, 64, 16),
    (64, 64, 4, 1, 4, 1, 2, 64, 16), (64, 64, 8, 1, 4, 1, 4, 64, 16), (128, 128, 4, 1, 4, 1, 4, 64, 16),
    (256, 128, 6, 1, 8, 1, 0, 32, 16), (256, 128, 6, 1, 8, 1, 8, 32, 16), (128, 64, 4, 1, 4, 1, 8, 64, 32),
    (256, 128, 3, 1, 8, 1, 8, 64, 32), (256, 256, 2, 1, 8, 1, 0, 64, 32),
})


def tg_built(plan) -> bool:
    """False for a plan tuple (bm, bn, stages, splits, ks, waves[, wk, loaders, sk, k depth, mfma, raster])
    whose kernel is pruned from the build."""
    p = tuple(plan) + (1, 0, 0, 64, 16)[max(0, len(plan) - 6):]
    return (p[0], p[1], p[2], p[4], p[5], p[6], p[7], p[9], p[10]) not in _TG_PRUNED


# one-split plans with a stream-K instantiation (csrc/kernels/tgemm.hip sk_plan, PLAIN epilogue only):
# (bm, bn, stages, ks, waves, loaders)
_SK_PLANS = {(64, 64, 3, 2, 4, 0), (64, 64, 4, 1, 4, 0), (64, 64, 4, 1, 4, 4), (64, 64, 4, 1, 4, 8),
             (64, 128, 3, 1, 8, 0), (128, 64, 4, 1, 4, 4)}
WS_FLOATS = 16 << 20      # 64 MiB of f32 split-K slabs per (device, owner)
WS_COUNTERS = 1 << 16

EPI_PLAIN, EPI_RESADD, EPI_QKV, EPI_SWIGLU, EPI_GELU = 0, 1, 2, 3, 4

# K-panel-major weight copies for the fused decoder GEMMs (GemmArgs.w_panel): every tgemm ring fill
# of the weight operand is one contiguous 1 KB instead of eight 128-B row pieces 4-11 KB apart
# (profiles/r3_decode_gemm_panel.md).  The row-major weight stays for the GEMV / skinny / hipBLASLt
# paths; models.llama keeps the panel copy only while both fit comfortably in HBM.
W_PANEL = True


def panel_weight(w: torch.Tensor) -> torch.Tensor:
    """[N, K] -> [K / 64, N, 64] (element (n, k) at ((k // 64) N + n) 64 + k % 64)."""
    N, K = w.shape
    return w.view(N, K // 64, 64).transpose(0, 1).contiguous()


def _nk(w: torch.Tensor) -> Tuple[int, int]:
    """(N, K) of a row-major [N, K] or panel [K / 64, N, 64] weight."""
    return (w.shape[1], w.shape[0] * 64) if w.dim() == 3 else (w.shape[0], w.shape[1])

_OWNER: contextvars.ContextVar = contextvars.ContextVar("dllm_gemm_ws_owner", default=None)


@contextlib.contextmanager
def workspace_owner(key):
    """Route split-K workspace lookups of this thread/context to ``key``'s own buffers."""
    tok = _OWNER.set(key)
    try:
        yield
    finally:
        _OWNER.reset(tok)


class _Planner:
    def __init__(self):
        self.plans: Dict[Tuple[int, int, int, bool], Tuple] = {}     # best overall, for linear()
        self.tg_plans: Dict[Tuple[int, int, int], Tuple] = {}        # best tgemm tile, for the fused ops
        self.fused_core: Dict[Tuple[int, int, int], str] = {}        # "tg" | "lin" | "gemvR" per tuned shape
        self.fused_opts: Dict[Tuple[int, int, int], Dict[str, float]] = {}   # measured us per core choice
        self.ws: Dict[Tuple, Tuple[torch.Tensor, torch.Tensor]] = {}
        self.sk_tables: Dict[Tuple, Tuple[torch.Tensor, int]] = {}   # stream-K segment lists per shape
        self.timings: Dict[Tuple[int, int, int, bool], Dict[str, float]] = {}

    def workspace(self, dev: torch.device, floats: int, tiles: int):
        """The fixed (part, counters) pair of the current owner on ``dev``; created once, outside
        capture, never grown."""
        if floats > WS_FLOATS or tiles > WS_COUNTERS:
            raise RuntimeError(f"split-K plan needs {floats} floats / {tiles} tickets > fixed workspace")
        key = (str(dev), _OWNER.get())
        w = self.ws.get(key)
        if w is None:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("split-K workspace first touched during graph capture (call reserve())")
            w = (torch.empty(WS_FLOATS, dtype=torch.float32, device=dev),
                 torch.zeros(WS_COUNTERS, dtype=torch.int32, device=dev))
            self.ws[key] = w
        return w


_P = _Planner()


def reserve(device) -> None:
    """Create the current owner's workspace on ``device`` (call before capturing graphs)."""
    _P.workspace(torch.device(device), 0, 0)


# ----------------------------------------------------------------------------- workspace needs

def _need(M: int, N: int, K: int, ntw: int, splits: int) -> Tuple[int, int]:
    nc = 16 * ntw
    tiles = (N + nc - 1) // nc
    kchunk = ((K + splits - 1) // splits + 31) // 32 * 32
    S = (K + kchunk - 1) // kchunk
    # split-K slabs are laid out with the kernel's row-tile height (MT x 16 rows, MT in 1/2/4/8)
    mp = 16 * (1 if M <= 16 else 2 if M <= 32 else 4 if M <= 64 else 8)
    return (S * tiles * nc * mp if S > 1 else 0), tiles


def _tg_splits(K: int, splits: int, ks: int = 1) -> int:
    q = 64 * ks
    kchunk = ((K + splits - 1) // splits + q - 1) // q * q
    return (K + kchunk - 1) // kchunk


def _need_tg(M: int, N: int, K: int, bm: int, bn: int, splits: int, ks: int = 1) -> Tuple[int, int]:
    tiles = ((M + bm - 1) // bm) * ((N + bn - 1) // bn)
    S = _tg_splits(K, splits, ks)
    return (S * tiles * bm * bn if S > 1 else 0), tiles


# ----------------------------------------------------------------------------- plans

def _heuristic(M: int, N: int, K: int) -> Tuple:
    if M > SKINNY_MAX_M:
        return ("blas",)
    ntw = 1 if M > 64 else 2
    tiles = (N + 16 * ntw - 1) // (16 * ntw)
    splits = max(1, min(16, math.ceil(512 / tiles), K // 256))
    return ("skinny", ntw, splits)


# Prefill-size buckets (M > MAX_M, PREFILL_TUNE): the fused ops' core is chosen per (bucket, N, K)
# between one tgemm launch with the epilogue fused and hipBLASLt + the standalone epilogue kernel;
# a prefill chunk uses the plan of the smallest bucket that holds it.  Rounds 4-5 measured it
# slower or neutral end to end (profiles/r4_prefill_gemm.md); with the grouped tile raster and the
# 8-loader 256 x 128 plans among the candidates (round 6) tgemm takes 8 of TinyLlama's 12 (bucket,
# shape) pairs (gate|up at 8K rows: 368 vs 448 us).  End to end it is within noise (+0.3 % over 7
# same-box arms of the driver command, prefill step time lower in 2 of 3; profiles/r6_prefill_core.md),
# and it is the default: the fused-epilogue kernel runs where it measured faster, hipBLASLt elsewhere.
PREFILL_MS = (2048, 4096, 8192)
PREFILL_TUNE = True
# decode buckets: the fused ops' core options are timed through the fused ops (_retime_fused)
FUSED_INSITU = True
# the split form (vendor / plain GEMM + standalone epilogue kernel) wins a fused op only when it is
# more than 3 % faster than the best one-launch core: on near-ties (QKV at the 512 bucket, 21-23 us
# either way in situ) the choice flipped run to run (profiles/r6_small_batch.md)
SPLIT_MARGIN = 1.03
# decode (v_new given): the standalone QKV epilogue hands V over row-major too, as the one-launch
# tgemm does, and the attention kernel writes the newest V^T (no 2-byte stores 32 B apart)
QKV_POST_VROWS = True
_PF_PLANS = ((256, 256, 2, 1, 1, 8), (256, 128, 3, 1, 1, 8), (192, 128, 3, 1, 1, 8), (128, 128, 3, 1, 1, 8),
             # 32-deep k-steps: 5-13 % ahead of the 64-deep tiles at 2-4K rows (profiles/r5_decode_gemm_lab.md)
             (256, 256, 4, 1, 1, 8, 1, 0, 0, 32),
             # grouped tile raster (plan element 12: m-tiles per group), the 8-loader 256 x 128 tile: the
             # fastest tgemm forms at 2-8K rows in scripts/exp/raster_probe.py (profiles/r6_gemm_fill_path.md)
             (256, 256, 2, 1, 1, 8, 1, 0, 0, 64, 16, 8), (256, 256, 4, 1, 1, 8, 1, 0, 0, 32, 16, 8),
             (256, 128, 3, 1, 1, 8, 1, 8, 0, 64, 16, 0), (256, 128, 3, 1, 1, 8, 1, 8, 0, 64, 16, 2),
             (256, 128, 3, 1, 1, 8, 1, 8, 0, 64, 16, 8))


def prefill_bucket(M: int) -> int:
    for b in PREFILL_MS:
        if M <= b:
            return b
    return PREFILL_MS[-1] if PREFILL_MS else M


def tg_plan(M: int, N: int, K: int) -> Tuple[int, ...]:
    """(bm, bn, stages, splits, ks, waves[, k-groups]) of the fused GEMM for this shape: tuned, else a
    heuristic sized so the grid covers the 256 CUs (bigger tiles first, split-K only for short
    grids)."""
    p = _P.tg_plans.get((M, N, K))
    if p is None and M > MAX_M and PREFILL_MS:
        p = _P.tg_plans.get((prefill_bucket(M), N, K))
    if p is not None:
        return tuple(p) + (1, 4)[len(p) - 4:] if len(p) < 6 else tuple(p)
    mt128, nt128 = -(-M // 128), -(-N // 128)
    if mt128 * nt128 >= 224:   # 8 waves: ~10 % ahead of 4 (profiles/r2_tgemm_tune_8b_shapes.log:25)
        return (128, 128, 3, 1, 1, 8)
    mt64, nt64 = -(-M // 64), -(-N // 64)
    if mt64 * nt128 >= 200:
        return (64, 128, 3, 1, 1, 4)
    tiles = mt64 * nt64
    splits = 1
    while tiles * splits * 2 <= 512 and K // (splits * 2) >= 256 and splits < 8:
        splits *= 2
    if _need_tg(M, N, K, 64, 64, splits)[0] > WS_FLOATS:
        splits = 1
    return (64, 64, 3, splits, 1, 4)


def tg_slots(M: int, N: int, K: int) -> int:
    """Row-sum-of-squares slots a RESADD GEMM of this shape writes (one per n-tile)."""
    return -(-N // tg_plan(M, N, K)[1])


def _run_plan(plan, x, w, swiglu, out, wp=None):
    if plan[0] == "blas":
        if swiglu:
            x = ref_silu_mul(x)
        return torch.matmul(x, w.t(), out=out) if out is not None else F.linear(x, w)
    ext = _native(x)
    if plan[0] == "tg":
        if swiglu:
            x = ref_silu_mul(x)
        y = out if out is not None else torch.empty((x.shape[0], w.shape[0]), dtype=x.dtype, device=x.device)
        _tgemm(ext, x, wp if wp is not None else w, EPI_PLAIN, plan[1:], y=y)
        return y
    if plan[0] == "gemv":
        y = out if out is not None else torch.empty((x.shape[0], w.shape[0]), dtype=x.dtype, device=x.device)
        ext.gemv(x, w, y, plan[1], swiglu)
        return y
    kind, ntw, splits = plan
    M, N, K = x.shape[0], w.shape[0], w.shape[1]
    y = out if out is not None else torch.empty((M, N), dtype=x.dtype, device=x.device)
    floats, tiles = _need(M, N, K, ntw, splits)
    part, cnt = _P.workspace(x.device, floats, tiles)
    ext.skinny_gemm(x, w, y, ntw, splits, swiglu, part, cnt)
    return y


def stream_k_table(M: int, N: int, K: int, bm: int, bn: int, ks: int, grid: int):
    """Stream-K work split of an (M, N, K) GEMM over ``grid`` workgroups (csrc/kernels/tgemm.hip,
    GemmArgs.sk_table): the tiles x k-steps iteration space is cut into ``grid`` equal contiguous
    ranges; workgroup w walks its range as segments (tile, first k-step, end k-step, slab index |
    contributors << 16).  A tile covered by c workgroups gets slab indices 0..c-1 in k order, so its
    last arriver sums the partials in the same order every time.  Returns (int32 [grid, segmax, 4]
    array padded with tile -1, cmax = the largest contributor count)."""
    import numpy as np
    mt, nt = -(-M // bm), -(-N // bn)
    tiles, nkt = mt * nt, K // (64 * ks)
    total = tiles * nkt
    segs = [[] for _ in range(grid)]
    contrib: Dict[int, list] = {}
    for w in range(grid):
        it, hi = w * total // grid, (w + 1) * total // grid
        while it < hi:
            t, kb = divmod(it, nkt)
            ke = min(nkt, kb + hi - it)
            segs[w].append([t, kb, ke, 0])
            contrib.setdefault(t, []).append((w, len(segs[w]) - 1))
            it += ke - kb
    cmax = max(len(v) for v in contrib.values())
    for t, lst in contrib.items():
        for idx, (w, j) in enumerate(lst):
            segs[w][j][3] = idx | (len(lst) << 16)
    segmax = max(1, max(len(s_) for s_ in segs))
    tab = np.full((grid, segmax, 4), -1, dtype=np.int32)
    for w, sl in enumerate(segs):
        if sl:
            tab[w, :len(sl)] = np.asarray(sl, dtype=np.int32)
    return tab, cmax


def _sk_grid(dev) -> int:
    return torch.cuda.get_device_properties(dev).multi_processor_count


def _sk_tensor(dev, M, N, K, bm, bn, ks):
    """The device copy of a stream-K table, created once per shape outside graph capture (the
    engine's capture warm-up runs every step eagerly first) and kept for the process lifetime."""
    key = (str(dev), M, N, K, bm, bn, ks)
    hit = _P.sk_tables.get(key)
    if hit is None:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("stream-K table first needed during graph capture (run the step eagerly first)")
        tab, cmax = stream_k_table(M, N, K, bm, bn, ks, _sk_grid(dev))
        hit = (torch.from_numpy(tab).to(dev), cmax)
        _P.sk_tables[key] = hit
    return hit


def _tgemm(ext, x, w, epi, plan, y=None, ssq_in=None, ssq_n=0, norm_scale=0.0, eps=0.0, ssq_out=None,
           pos=None, cos_sin=None, slots=None, q_out=None, kc=None, vc=None, nq=0, nkv=0, d=0, bias=None,
           v_rows=None):
    """plan = (bm, bn, stages, splits[, ks, waves[, k-groups[, loader waves[, stream-K[, k depth[, mfma[, raster]]]]]]])"""
    bm, bn, st, sp = plan[:4]
    ks, nw = (plan[4], plan[5]) if len(plan) >= 6 else (1, 4)
    wk = plan[6] if len(plan) >= 7 else 1
    nl = plan[7] if len(plan) >= 8 else 0
    sk = len(plan) >= 9 and plan[8] == 1
    bk = plan[9] if len(plan) >= 10 else 64
    mf = plan[10] if len(plan) >= 11 else 16
    raster = plan[11] if len(plan) >= 12 else 0
    if sk and epi != EPI_PLAIN:
        raise ValueError("tgemm: stream-K plans are built for the PLAIN epilogue only")
    M = x.shape[0]
    N, K = _nk(w)
    if K % (64 * ks):
        ks, wk = 1, 1
    part = cnt = tab = None
    cmax = 0
    if sk:
        tab, cmax = _sk_tensor(x.device, M, N, K, bm, bn, ks)
        tiles = -(-M // bm) * -(-N // bn)
        part, cnt = _P.workspace(x.device, tiles * cmax * bm * bn, tiles)
        sp = 1
    elif _tg_splits(K, sp, ks) > 1:
        floats, tiles = _need_tg(M, N, K, bm, bn, sp, ks)
        part, cnt = _P.workspace(x.device, floats, tiles)
    ext.tgemm(x, w, y, epi, bm, bn, st, sp, ks, nw, part, cnt, ssq_in, int(ssq_n), float(norm_scale), float(eps), ssq_out,
              pos, cos_sin, slots, q_out, kc, vc, int(nq), int(nkv), int(d), bias, int(wk), int(nl), tab, int(cmax),
              v_rows, int(bk), int(mf), int(raster))


def ref_silu_mul(gu):
    from . import silu_mul
    return silu_mul(gu)


def _key(x, w, swiglu):
    return (x.shape[0], w.shape[0], w.shape[1], bool(swiglu))


def linear(x: torch.Tensor, w: torch.Tensor, out: Optional[torch.Tensor] = None,
           wp: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``x @ w.T`` on the shape's tuned plan; ``wp``: the panel copy a tgemm plan streams."""
    if not x.is_cuda or os.environ.get("DLLM_GEMM") == "blas":
        return F.linear(x, w) if out is None else torch.matmul(x, w.t(), out=out)
    plan = _P.plans.get(_key(x, w, False))
    if plan is None:
        if x.shape[0] > MAX_M:
            plan = ("blas",)
        else:
            plan = _heuristic(x.shape[0], w.shape[0], w.shape[1])
    return _run_plan(plan, x, w, False, out, wp)


def norm_linear(h: torch.Tensor, residual: torch.Tensor, spare: torch.Tensor, norm_w: torch.Tensor, eps: float,
                w: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """``linear(rmsnorm(h + residual) * norm_w, w)`` and the updated residual stream (unfused
    layer path: tensor parallel, CPU).  (A one-launch GEMV form, gemv.hip NORM, measured SLOWER at
    batch 1, profiles/r1_small_batch_decode.md; ``spare`` is kept for that interface.)"""
    from . import rms_norm
    x = rms_norm(h, norm_w, eps, residual=residual)
    return linear(x, w), residual


def linear_swiglu(gu: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """``silu(gate) * up @ w.T`` with gu = [gate | up] of width 2K."""
    if not gu.is_cuda:
        return F.linear(ref.silu_mul(gu), w)
    if gu.shape[0] > MAX_M or os.environ.get("DLLM_GEMM") == "blas":
        from . import silu_mul
        return linear(silu_mul(gu), w)
    plan = _P.plans.get(_key(gu, w, True)) or _heuristic(gu.shape[0], w.shape[0], w.shape[1])
    return _run_plan(plan, gu, w, True, None)


# ----------------------------------------------------------------------------- fused decoder ops
#
# Two implementations of each fused op: the tgemm epilogue (one launch), or the shape's best plain
# GEMM (GEMV / skinny / hipBLASLt, whatever the autotuner picked for linear()) followed by the same
# epilogue as a standalone kernel (qkv_post / res_add_ssq / swiglu_post).
# The autotuner records, per decode bucket and shape, which is faster (the standalone epilogue
# is charged its measured time, _post_us; POST_US only where it cannot be measured); shapes it never saw (prefill chunks above MAX_M) use the vendor core,
# which wins at large M (profiles/r2_tgemm_tune.md).
POST_US = 3.0


def use_vendor_core(M: int, N: int, K: int) -> bool:
    """True: run the fused op as ``linear()`` (the shape's best plain plan — GEMV / skinny /
    hipBLASLt / plain tgemm) followed by the standalone epilogue kernel; False: one tgemm launch
    with the epilogue fused.  (A ``gemvR`` choice is taken before this by ``fused_gemv_r``.)"""
    env = os.environ.get("DLLM_FUSED_CORE")
    if env in ("tg", "blas", "lin"):
        return env != "tg"
    c = _P.fused_core.get((M, N, K))
    if c is None and M > MAX_M and PREFILL_MS:
        c = _P.fused_core.get((prefill_bucket(M), N, K))
    if c is not None:
        return c != "tg"
    return M > MAX_M


def fused_gemv_r(x: torch.Tensor, N: int) -> int:
    """R (output rows per wave) of the fused-epilogue GEMV (csrc/kernels/gemv.hip EPI) if the
    autotuner picked it for this fused op's shape (``fused_core`` = ``gemvR``; forced by
    ``DLLM_FUSED_CORE=gemvR``), else 0.  Batch <= 8 only: it replaces GEMV/skinny + a standalone
    epilogue launch (qkv_post / res_add_ssq / swiglu_post) with one launch."""
    M, K = x.shape[0], x.shape[1]
    if M not in _GEMV_MS or K % 8 or M * K * 2 > 64 * 1024 or x.stride(1) != 1 or x.stride(0) % 8 or N % 32:
        return 0
    env = os.environ.get("DLLM_FUSED_CORE")
    c = env if env else _P.fused_core.get((M, N, K))
    if isinstance(c, str) and c.startswith("gemv") and c[4:] in ("1", "2", "4"):
        return int(c[4:])
    return 0


def fused_ske(x: torch.Tensor, N: int, K: int) -> int:
    """Split count of the small-batch fused-epilogue MFMA GEMM (skinny_epi, 32-column tiles) if the
    autotuner picked it for this fused op's shape (``fused_core`` = ``skE<splits>``; forced by
    ``DLLM_FUSED_CORE=skE<splits>``), else 0."""
    M = x.shape[0]
    if not (0 < M <= SKE_MAX_M) or K % 64 or N % 32 or x.stride(1) != 1 or x.stride(0) % 8:
        return 0
    env = os.environ.get("DLLM_FUSED_CORE")
    c = env if env and env.startswith("skE") else _P.fused_core.get((M, N, K))
    if isinstance(c, str) and c.startswith("skE") and c[3:].isdigit():
        return int(c[3:])
    return 0


def _ske_ws(x: torch.Tensor, N: int, K: int, splits: int):
    tiles = -(-N // 32)
    kchunk = ((-(-K // splits)) + 31) // 32 * 32
    S = -(-K // kchunk)
    return _P.workspace(x.device, (S * tiles * 32 * 16) if S > 1 else 0, tiles)


def skinny_epi(x: torch.Tensor, w: torch.Tensor, epi: int, splits: int, y=None, res=None, ssq_out=None, ssq_in=None,
               ssq_n: int = 0, scale: float = 0.0, eps: float = 0.0, pos=None, cos_sin=None, slots=None, q_out=None,
               kc=None, vc=None, nq: int = 0, nkv: int = 0, d: int = 0) -> int:
    """One launch of the small-batch fused-epilogue GEMM (``w`` row-major or the panel copy)."""
    N, K = _nk(w)
    part, cnt = _ske_ws(x, N, K, splits)
    return int(_native(x).skinny_epi(x, w, y, 2, int(splits), int(epi), part, cnt, res, ssq_out, ssq_in, int(ssq_n),
                                     float(scale), float(eps), pos, cos_sin, slots, q_out, kc, vc, int(nq), int(nkv),
                                     int(d)))


def _core(x: torch.Tensor, w: torch.Tensor, wp: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Plain product for the split (core + epilogue) form of a fused op: the tuned plan of this
    shape (M <= MAX_M), hipBLASLt above."""
    return linear(x, w, wp=wp) if x.shape[0] <= MAX_M else F.linear(x, w)

def qkv_rope_cache(r: torch.Tensor, w: torch.Tensor, ssq: torch.Tensor, ssq_n: int, eps: float,
                   positions: torch.Tensor, cos_sin: torch.Tensor, slots: torch.Tensor, k_cache: torch.Tensor,
                   v_cache: torch.Tensor, nq: int, nkv: int, d: int, wp: Optional[torch.Tensor] = None,
                   v_new: Optional[torch.Tensor] = None):
    """q [T, nq, d] of ``rope(rmsnorm(r) . Wqkv^T)``, K/V written to the paged caches, one launch.

    ``w`` is the folded/permuted weight of models.llama.fuse_qkv_weight; ``ssq[:ssq_n]`` holds
    the partial row sums of r^2 written by the producer of ``r``.

    ``v_new`` ([T, nkv * d], decode steps only): where the one-launch GEMM runs, V is written there
    row-major instead of into the V^T cache, and the decode attention kernel moves each sequence's
    newest V into the cache itself (``paged_attention(v_new=...)``: the GEMM's V-column workgroups
    were its stragglers, profiles/r5_qkv_epilogue.md).  Returns ``(q, v_new or None)`` then — None
    where another implementation ran and the cache already holds V."""
    T, H = r.shape
    q = torch.empty((T, nq, d), dtype=r.dtype, device=r.device)
    if T == 0:
        return q if v_new is None else (q, None)
    out = (lambda used: q if v_new is None else (q, v_new if used else None))
    R = fused_gemv_r(r, w.shape[0])
    if R:
        _native(r).gemv_qkv(r, w, ssq, int(ssq_n), 1.0 / H, float(eps), positions, cos_sin, slots, q, k_cache,
                            v_cache, nq, nkv, d, R)
        return out(False)
    sp = fused_ske(r, w.shape[0], H)
    if sp:
        skinny_epi(r, wp if wp is not None else w, EPI_QKV, sp, ssq_in=ssq, ssq_n=ssq_n, scale=1.0 / H, eps=eps,
                   pos=positions, cos_sin=cos_sin, slots=slots, q_out=q, kc=k_cache, vc=v_cache, nq=nq, nkv=nkv, d=d)
        return out(False)
    if use_vendor_core(T, w.shape[0], H):
        vr = v_new if QKV_POST_VROWS else None
        _native(r).qkv_post(_core(r, w, wp), ssq, int(ssq_n), 1.0 / H, float(eps), positions, cos_sin, slots, q,
                            k_cache, v_cache, nq, nkv, d, vr)
        return out(vr is not None)
    _tgemm(_native(r), r, wp if wp is not None else w, EPI_QKV, tg_plan(T, w.shape[0], H), ssq_in=ssq, ssq_n=ssq_n, norm_scale=1.0 / H,
           eps=eps, pos=positions, cos_sin=cos_sin, slots=slots, q_out=q, kc=k_cache, vc=v_cache, nq=nq, nkv=nkv,
           d=d, v_rows=v_new)
    return out(True)


def matmul_resadd(x: torch.Tensor, w: torch.Tensor, residual: torch.Tensor, ssq_out: torch.Tensor,
                  wp: Optional[torch.Tensor] = None) -> int:
    """``residual += x . w^T`` (bf16 rounding as ``rms_norm``'s residual add) and the partial row
    sums of the new residual's squares into ``ssq_out[:slots]``; returns ``slots``."""
    M, N, K = x.shape[0], w.shape[0], w.shape[1]
    R = fused_gemv_r(x, N) if M else 0
    if R:
        return int(_native(x).gemv_resadd(x, w, residual, ssq_out, R))
    sp = fused_ske(x, N, K) if M else 0
    if sp:
        return skinny_epi(x, wp if wp is not None else w, EPI_RESADD, sp, res=residual, ssq_out=ssq_out)
    if M and use_vendor_core(M, N, K):
        return int(_native(x).res_add_ssq(_core(x, w, wp), residual, ssq_out))
    plan = tg_plan(M, N, K)
    if M:
        _tgemm(_native(x), x, wp if wp is not None else w, EPI_RESADD, plan, y=residual, ssq_out=ssq_out)
    return -(-N // plan[1])


def swiglu_matmul(r: torch.Tensor, w: torch.Tensor, ssq: torch.Tensor, ssq_n: int, eps: float,
                  wp: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``silu(g) * u`` with ``[g | u] = rmsnorm(r) . Wgu^T`` (interleaved rows, models.llama
    .fuse_gate_up_weight) -> [T, I]."""
    T, H = r.shape
    act = torch.empty((T, w.shape[0] // 2), dtype=r.dtype, device=r.device)
    R = fused_gemv_r(r, w.shape[0]) if T else 0
    if R:
        _native(r).gemv_swiglu(r, w, ssq, int(ssq_n), 1.0 / H, float(eps), act, R)
        return act
    sp = fused_ske(r, w.shape[0], H) if T else 0
    if sp:
        skinny_epi(r, wp if wp is not None else w, EPI_SWIGLU, sp, y=act, ssq_in=ssq, ssq_n=ssq_n, scale=1.0 / H,
                   eps=eps)
        return act
    if T and use_vendor_core(T, w.shape[0], H):
        _native(r).swiglu_post(_core(r, w, wp), ssq, int(ssq_n), 1.0 / H, float(eps), act)
        return act
    if T:
        _tgemm(_native(r), r, wp if wp is not None else w, EPI_SWIGLU, tg_plan(T, w.shape[0], H), y=act, ssq_in=ssq, ssq_n=ssq_n,
               norm_scale=1.0 / H, eps=eps)
    return act


def res_add_ssq(h: Optional[torch.Tensor], r: torch.Tensor, ssq: torch.Tensor) -> int:
    """``r += h`` in place (h may be None) and the row sums of ``r^2``: ``ssq`` [M] gets the full
    sum, ``ssq`` [slots, >= M] partial sums over column slices.  Returns the slots written."""
    return int(_native(r).res_add_ssq(h, r, ssq))


# ----------------------------------------------------------------------------- encoder (bias) ops

def _enc_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    return x.is_cuda and w.shape[1] % 64 == 0 and w.shape[0] % 8 == 0 and x.stride(1) == 1 and x.stride(0) % 8 == 0


def linear_bias(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, gelu: bool = False) -> torch.Tensor:
    """``x . w^T + bias`` (optionally followed by erf-GELU) in one tgemm launch (bias / GELU
    epilogue): the router encoder's QKV and FFN-up projections."""
    if not _enc_ok(x, w):
        y = F.linear(x, w, bias)
        return ref.gelu(y) if gelu else y
    M, N, K = x.shape[0], w.shape[0], w.shape[1]
    y = torch.empty((M, N), dtype=x.dtype, device=x.device)
    if M:
        _tgemm(_native(x), x, w, EPI_GELU if gelu else EPI_PLAIN, tg_plan(M, N, K), y=y, bias=bias)
    return y


def linear_bias_residual(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, residual: torch.Tensor) -> torch.Tensor:
    """``residual += x . w^T + bias`` in place (tgemm residual epilogue with bias; bf16 rounding of
    the projection before the add, as F.linear followed by an add); returns ``residual``."""
    if not _enc_ok(x, w):
        residual.copy_((F.linear(x, w, bias).float() + residual.float()).to(residual.dtype))
        return residual
    M, N, K = x.shape[0], w.shape[0], w.shape[1]
    if M:
        _tgemm(_native(x), x, w, EPI_RESADD, tg_plan(M, N, K), y=residual, bias=bias)
    return residual


def max_slots(N: int, M: int = 0) -> int:
    """Rows a partial-row-sum buffer needs for a residual producer of N columns: one per 64-column
    tgemm tile, at batch <= 8 one per fused-GEMV workgroup (N / 4 at R = 1), at batch <= 16 one
    per 32-column small-batch MFMA tile (skinny_epi)."""
    if 0 < M <= max(_GEMV_MS):
        return -(-N // 4)
    return -(-N // 32) if 0 < M <= SKE_MAX_M else -(-N // 64)


# ----------------------------------------------------------------------------- autotuning

def _time(fn, iters=24) -> float:
    """GPU time per call of fn(i) in us, measured as a hipGraph replay of ``iters`` calls (the
    decode step is a graph replay too, so host launch cost is excluded exactly as in serving).
    Callers rotate operands over i so weights come from HBM, not the 256 MiB Infinity Cache."""
    fn(0)  # eager warm-up: initialises libraries outside capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        with torch.cuda.graph(g, stream=st):
            for i in range(iters):
                fn(i)
    torch.cuda.current_stream().wait_stream(st)
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / iters


def _post_us(M: int, N: int, dev) -> float:
    """Measured cost of the standalone epilogue a vendor-core fused op adds: one pass reading two
    [M, N] bf16 operands and writing one (res_add_ssq; qkv_post / swiglu_post move the same or
    fewer bytes).  Charged to hipBLASLt when choosing the fused op's core."""
    if N % 8:
        return POST_US
    y = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
    r = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
    ssq = torch.empty(max_slots(N), M, dtype=torch.float32, device=dev)
    ext = _native(y)
    return _time(lambda i: ext.res_add_ssq(y, r, ssq))


def _plan_key(k) -> str:
    if len(k) == 3:
        return "t,%d,%d,%d" % k
    return "%d,%d,%d,%d" % (k[0], k[1], k[2], int(k[3]))


def autotune(shapes: Iterable[Tuple[int, int, bool]], ms: Iterable[int], device, verbose: bool = False,
             fused: Iterable[Tuple[int, int]] = (), prefill: bool = False, qkv_dims=None, qkv_cache=None) -> None:
    """Measure every candidate plan for each (M, N, K, swiglu) and keep the fastest.

    ``fused``: the (N, K) shapes of one decoder layer's fused ops (QKV, Wo, gate|up, down); a
    residual producer keeps the fused GEMV only where its consumer runs it too
    (``_couple_gemv_choices``).  Their fused-op cores are timed through the fused ops themselves
    (``_retime_fused``); ``qkv_dims`` = (nq, nkv, d) of the QKV op (None: QKV keeps the stand-in
    timings); ``qkv_cache`` = one layer's (K, V^T) caches of the engine, which the QKV timing writes
    into at scattered free blocks (the TLB reach of a whole serving pool, not of a small buffer)."""
    dev = torch.device(device)
    if dev.type != "cuda" or os.environ.get("DLLM_GEMM") == "blas":
        return
    reserve(dev)
    cache = os.environ.get("DLLM_GEMM_PLANS")  # JSON plan cache: re-use a previous run's choices
    if cache and os.path.exists(cache):
        import json
        with open(cache) as f:
            for k, v in json.load(f).items():
                parts = k.split(",")
                if parts[0] == "t":
                    _P.tg_plans[(int(parts[1]), int(parts[2]), int(parts[3]))] = tuple(v)
                elif parts[0] == "c":
                    _P.fused_core[(int(parts[1]), int(parts[2]), int(parts[3]))] = v
                else:
                    _P.plans[(int(parts[0]), int(parts[1]), int(parts[2]), parts[3] == "1")] = tuple(v)
    shapes = list(shapes)
    fused = list(fused)
    # the fused ops' tgemm plans stream the panel weight copies: time them in that layout
    roles = {}
    if len(fused) == 4:   # (QKV, Wo, gate|up, down) of a dense layer
        roles = {tuple(fused[0]): "qkv", tuple(fused[1]): "resadd", tuple(fused[2]): "swiglu",
                 tuple(fused[3]): "resadd"}
    _autotune(shapes, list(ms), dev, verbose, {tuple(f) for f in fused} if W_PANEL else set(), roles, qkv_dims,
              qkv_cache)
    _couple_gemv_choices(fused, list(ms), verbose)
    if PREFILL_TUNE or prefill:
        _autotune_prefill(fused, dev, verbose)
    if cache:
        import json
        d = {_plan_key(k): list(v) for k, v in _P.plans.items()}
        d.update({_plan_key(k): list(v) for k, v in _P.tg_plans.items()})
        d.update({"c,%d,%d,%d" % k: v for k, v in _P.fused_core.items()})
        if os.path.dirname(cache):
            os.makedirs(os.path.dirname(cache), exist_ok=True)
        with open(cache, "w") as f:
            json.dump(d, f)


def _autotune_prefill(fused, dev, verbose: bool) -> None:
    """Fused-op core at the prefill buckets: one tgemm launch with the epilogue fused (PLAIN timed,
    the fused epilogues write the same tile or less) against hipBLASLt + the standalone epilogue
    kernel; the tgemm plans stream the K-panel weight copy the model keeps (W_PANEL)."""
    for (N, K) in {tuple(f) for f in fused}:
        todo = [M for M in PREFILL_MS if (M, N, K) not in _P.fused_core]
        if not todo or K % 64:
            continue
        copies = max(2, min(8, (256 << 20) // (N * K * 2)))
        ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(copies)]
        wps = [panel_weight(w) for w in ws] if W_PANEL else ws
        for M in todo:
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            y = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            ext = _native(x)
            lin = _time(lambda i: torch.matmul(x, ws[i % copies].t(), out=y), iters=8) + _post_us(M, N, dev)
            best, best_t = None, float("inf")
            for p in _PF_PLANS:
                try:
                    t = _time(lambda i: _tgemm(ext, x, wps[i % copies], EPI_PLAIN, p, y=y), iters=8)
                except Exception:  # noqa: BLE001 - plan refused for this shape
                    continue
                if t < best_t:
                    best, best_t = p, t
            if best is not None:
                _P.tg_plans[(M, N, K)] = best
            _P.fused_core[(M, N, K)] = "tg" if best is not None and best_t < lin else "lin"
            if verbose:
                print(f"gemm prefill M={M} N={N} K={K}: blas+post {lin:.1f}us, tgemm {best} {best_t:.1f}us "
                      f"-> {_P.fused_core[(M, N, K)]}", flush=True)
            del x, y
        del ws, wps


def _couple_gemv_choices(fused, ms, verbose: bool) -> None:
    """A fused-GEMV residual producer leaves one row-sum slot per workgroup (hundreds), which a
    GEMV consumer sums in one round trip but a tgemm prologue or standalone epilogue walks
    serially.  ``fused`` = (QKV, Wo, gate|up, down) shapes of a dense layer: Wo feeds gate|up and
    down feeds the next layer's QKV, so a producer keeps the GEMV only if its consumer runs it too
    (MoE layers pass (QKV, Wo): their producers feed standalone norms, no constraint)."""
    fused = list(fused)
    pairs = [(fused[1], fused[2]), (fused[3], fused[0])] if len(fused) == 4 else []
    for M in ms:
        for prod, cons in pairs:
            kp, kc = (M,) + tuple(prod), (M,) + tuple(cons)
            cp, cc = _P.fused_core.get(kp), _P.fused_core.get(kc)
            if cp is None or not cp.startswith("gemv") or (cc is not None and cc.startswith(("gemv", "skE"))):
                continue
            opts = {c: t for c, t in _P.fused_opts.get(kp, {}).items() if not c.startswith("gemv")}
            _P.fused_core[kp] = min(opts, key=opts.get) if opts else "lin"
            if verbose:
                print(f"gemm M={M} N={kp[1]} K={kp[2]}: fused GEMV dropped (its consumer N={kc[1]} K={kc[2]} "
                      f"runs {cc}, which would walk the per-workgroup row sums) -> core {_P.fused_core[kp]}",
                      flush=True)


def _tg_cands(M: int, N: int, K: int):
    if K % 64:
        return []
    out = []
    for bm, bn, nw in _TG_TILES:
        if (bm == 128 and M <= 64) or (bm >= 192 and M <= 128):
            continue
        tiles = -(-M // bm) * -(-N // bn)
        for ks in (1, 2):
            if K % (64 * ks):
                continue
            for sp in _TG_SPLITS:
                if sp > 1 and (K // sp < 256 * ks or tiles * sp > 2048):
                    continue
                if _tg_splits(K, sp, ks) != sp:
                    continue
                if _need_tg(M, N, K, bm, bn, sp, ks)[0] > WS_FLOATS:
                    continue
                for st in ((2, 3, 4, 6) if bm <= 128 and ks == 1 else (2, 3)):
                    if st * ks * (bm + bn) * 128 > 150 * 1024:
                        continue   # the ring would not fit the LDS
                    out.append((bm, bn, st, sp, ks, nw))
                    if ks == 2 and nw == 4 and st <= 3 and bm <= 128 and bn <= 128:
                        out.append((bm, bn, st, sp, ks, nw, 2))   # two k-groups of 4 waves
    if N % 8 == 0:
        for bm, bn, nw, st, nl, m_min in _TG_NL:
            if M < m_min or (bm == 16 and M > 16):
                continue
            tiles = -(-M // bm) * -(-N // bn)
            for sp in (1, 2, 3, 4):
                if sp > 1 and (K // sp < 256 or tiles * sp > 2048 or _tg_splits(K, sp) != sp):
                    continue
                if _need_tg(M, N, K, bm, bn, sp)[0] > WS_FLOATS:
                    continue
                out.append((bm, bn, st, sp, 1, nw, 1, nl))
    # 32 x 32 x 16 MFMA forms of the flagship's tiles, with the splits their 16 x 16 forms take
    if N % 8 == 0:
        for p in _TG_M32:
            bm, bn, st, _, ks, nw, wk, nl = p[:8]
            if (bm >= 128 and M <= 64) or (bm == 256 and M <= 128) or K % (64 * ks):
                continue
            tiles = -(-M // bm) * -(-N // bn)
            for sp in (1, 2, 3, 4):
                if sp > 1 and (K // sp < 256 * ks or tiles * sp > 2048 or _tg_splits(K, sp, ks) != sp):
                    continue
                if _need_tg(M, N, K, bm, bn, sp, ks)[0] > WS_FLOATS:
                    continue
                out.append((bm, bn, st, sp) + tuple(p[4:]))
    # Stream-K forms (one workgroup per CU walking equal shares of tiles x k-steps, _SK_PLANS) are not
    # offered: measured, they never beat the one-unit plans on the TinyLlama shapes at M = 320-448,
    # because the shared-operand L2 -> LDS traffic, not the idle CUs, sets the time
    # (profiles/r3_decode_gemm_panel.md section 5).  They stay built for the PLAIN epilogue (tests).
    return [c for c in out if tg_built(c)]


def _retime_fused(tkey, role, opts, x, ws, wps, qkv_dims, dev, qkv_cache=None):
    """Time every fused-core option of a decoder-layer shape through the fused op itself: its real
    epilogue and its row-scale prologue over the producer's partial row sums.  The stand-in timings
    (PLAIN tgemm, RESADD GEMV / skinny_epi) missed those: gate|up at batch 4 chose a tgemm timed at
    13.6 us that ran 17.3 us inside the step graph (profiles/r6_small_batch.md)."""
    M, N, K = tkey
    copies = len(ws)
    wsrc = lambda i: (ws[i % copies], wps[i % copies] if wps is not None else None)
    slots_in = -(-K // 32)   # the producer's partial row sums (as many as a skinny_epi producer leaves)
    ssq = torch.rand(slots_in, M, device=dev) + 1.0
    if role == "resadd":
        res = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
        so = torch.empty(max_slots(N, M), M, dtype=torch.float32, device=dev)
        fn = lambda i: matmul_resadd(x, wsrc(i)[0], res, so, wp=wsrc(i)[1])
    elif role == "swiglu":
        fn = lambda i: swiglu_matmul(x, wsrc(i)[0], ssq, slots_in, 1e-5, wp=wsrc(i)[1])
    elif role == "qkv" and qkv_dims is not None:
        nq, nkv, d = qkv_dims
        if (nq + 2 * nkv) * d != N:
            return None
        # the step writes each row's K / V into its own block of a large pool: scattered slots in the
        # engine's own cache (else a 64 MiB pool; contiguous slots in a tiny cache timed the split
        # form's K / V^T writes 3.5 us per call faster than they run in the flagship's step)
        if (qkv_cache is not None and tuple(qkv_cache[0].shape[1:]) == (nkv, 16, d)
                and qkv_cache[0].shape[0] >= M + 1):
            kc, vc = qkv_cache
            nblk = kc.shape[0]
        else:
            nblk = max(-(-M // 16) + 1, (64 << 20) // (nkv * 16 * d * 2))
            kc = torch.zeros(nblk, nkv, 16, d, dtype=torch.bfloat16, device=dev)
            vc = torch.zeros(nblk, nkv, d, 16, dtype=torch.bfloat16, device=dev)
        pos = torch.randint(100, 4000, (M,), dtype=torch.int32, device=dev)
        sl = (torch.randperm(nblk, device=dev)[:M] * 16 + torch.randint(0, 16, (M,), device=dev)).to(torch.int32)
        cs = torch.rand(4096, d, device=dev)
        # (d = 64 decode hands V over row-major, as models.llama does: the one-launch cores then skip
        # the strided V^T cache writes)
        vn = torch.empty(M, nkv * d, dtype=torch.bfloat16, device=dev) if d == 64 else None
        fn = lambda i: qkv_rope_cache(x, wsrc(i)[0], ssq, slots_in, 1e-5, pos, cs, sl, kc, vc, nq, nkv, d,
                                      wp=wsrc(i)[1], v_new=vn)
    else:
        return None
    saved = _P.fused_core.get(tkey)
    out = {}
    try:
        for _ in range(2):   # two interleaved passes, the faster of each option's two times
            for opt in opts:
                _P.fused_core[tkey] = opt
                try:
                    t = _time(fn)
                except Exception:  # noqa: BLE001 - option not runnable for this shape
                    t = float("inf")
                out[opt] = min(out.get(opt, float("inf")), t)
    finally:
        if saved is None:
            _P.fused_core.pop(tkey, None)
        else:
            _P.fused_core[tkey] = saved
    return out


def _autotune(shapes, ms, dev, verbose: bool, panel_shapes=frozenset(), roles=None, qkv_dims=None,
              qkv_cache=None) -> None:
    use_tg = True
    for (N, K, sw) in shapes:
        copies = max(2, min(64, math.ceil((768 << 20) / (N * K * 2))))
        ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(copies)]
        wps = [panel_weight(w) for w in ws] if (N, K) in panel_shapes and K % 64 == 0 and not sw else None
        for M in ms:
            if M > MAX_M:
                continue
            key = (M, N, K, sw)
            tkey = (M, N, K)
            need_plain = key not in _P.plans
            need_tg = use_tg and not sw and (tkey not in _P.tg_plans or tkey not in _P.fused_core) and K % 64 == 0
            if not (need_plain or need_tg):
                continue
            x = torch.randn(M, 2 * K if sw else K, device=dev).to(torch.bfloat16)
            cands = [("blas",)]
            if M in _GEMV_MS and K % 8 == 0 and M * K * 2 <= 64 * 1024:
                cands.extend(("gemv", r) for r in _GEMV_RS)
            for ntw in (_NTWS if M <= SKINNY_MAX_M else ()):
                if M > 64 and ntw == 4:
                    continue
                for s in _SPLITS:
                    if s > 1 and K // s < 128:
                        continue
                    floats, tiles = _need(M, N, K, ntw, s)
                    if floats > WS_FLOATS or tiles > WS_COUNTERS:
                        continue
                    cands.append(("skinny", ntw, s))
            if use_tg and not sw:
                cands.extend(("tg",) + c for c in _tg_cands(M, N, K))
            res = {}
            for c in cands:
                res[c] = _time(lambda i: _run_plan(c, x, ws[i % copies], sw, None,
                                                   wps[i % copies] if wps is not None else None))
            best = min(res, key=res.get)
            if need_plain:
                _P.plans[key] = best
                _P.timings[key] = {str(c): round(t, 2) for c, t in res.items()}
            tgc = [c for c in res if c[0] == "tg"]
            post = None
            if need_tg and tgc:
                best_tg = min(tgc, key=res.get)
                _P.tg_plans[tkey] = best_tg[1:]
                post = _post_us(M, N, dev)
                # the split form runs the shape's best plain plan (GEMV at M <= 8, skinny, ...)
                best_plain = min(res[c] for c in res if c[0] != "tg")
                opts = {"tg": res[best_tg], "lin": best_plain + post}
                # fused-epilogue GEMV (one launch): timed in its RESADD form (the paired QKV /
                # SwiGLU forms stream the same rows with the same per-wave loads)
                gv = [c for c in res if c[0] == "gemv"]
                if gv and N % 32 == 0:
                    ext = _native(x)
                    rr = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
                    sq = torch.empty(max_slots(N, M), M, dtype=torch.float32, device=dev)
                    for c in gv:
                        opts["gemv%d" % c[1]] = _time(lambda i: ext.gemv_resadd(x, ws[i % copies], rr, sq, c[1]))
                # small-batch MFMA GEMM with the epilogue fused (one launch), timed in its RESADD form
                # on the weight layout the fused ops stream (the panel copy where the model keeps one)
                if M <= SKE_MAX_M and N % 32 == 0 and K % 64 == 0:
                    rr = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
                    sq = torch.empty(max_slots(N, M), M, dtype=torch.float32, device=dev)
                    src = wps if wps is not None else ws
                    for sp in _SKE_SPLITS:
                        if sp > 1 and K // sp < 256:
                            continue
                        try:
                            opts["skE%d" % sp] = _time(lambda i: skinny_epi(x, src[i % copies], EPI_RESADD, sp, res=rr,
                                                                             ssq_out=sq))
                        except Exception:  # noqa: BLE001 - workspace / shape refused
                            pass
                role = (roles or {}).get((N, K))
                if FUSED_INSITU and role is not None and M <= MAX_M and os.environ.get("DLLM_FUSED_CORE") is None:
                    insitu = _retime_fused(tkey, role, opts, x, ws, wps, qkv_dims, dev, qkv_cache)
                    if insitu:
                        opts = insitu
                core = min(opts, key=opts.get)
                one = {c: t for c, t in opts.items() if c != "lin"}
                if core == "lin" and one and min(one.values()) <= SPLIT_MARGIN * opts["lin"]:
                    core = min(one, key=one.get)
                _P.fused_core[tkey] = core
                _P.fused_opts[tkey] = opts
            if verbose:
                bk = {k: min((c for c in res if c[0] == k), key=res.get, default=None)
                      for k in ("gemv", "skinny", "tg")}
                extra = " ".join(f"{k}={c[1:]}:{res[c]:.1f}us" for k, c in bk.items() if c)
                top = sorted(tgc, key=res.get)[:4]
                extra += " | tg top: " + " ".join(f"{c[1:]}:{res[c]:.1f}" for c in top)
                if post is not None:
                    extra += (f" | post {post:.1f}us | fused " +
                              " ".join(f"{k}:{v:.1f}" for k, v in _P.fused_opts[tkey].items()) +
                              f" -> core {_P.fused_core[tkey]}")
                print(f"gemm M={M} N={N} K={K} swiglu={sw}: best={best} {res[best]:.1f}us "
                      f"({N * K * 2 / res[best] / 1e3:.0f} GB/s, {2 * M * N * K / res[best] / 1e6:.0f} TF/s; "
                      f"blas {res[('blas',)]:.1f}us; {extra})", flush=True)
        del ws, wps


def plans() -> Dict:
    d = {str(k): v for k, v in _P.plans.items()}
    d.update({"tg" + str(k): v for k, v in _P.tg_plans.items()})
    return d
