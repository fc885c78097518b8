"""Linear layers: decode-shaped GEMMs on the hand-written MFMA skinny kernel, autotuned.

``linear(x, w)`` computes ``x @ w.T`` (w stored [N, K], K contiguous).
``linear_swiglu(gu, w)`` computes ``silu(gu[:, :K]) * gu[:, K:] @ w.T`` — the SwiGLU activation is
fused into the down projection's operand load, so decode runs no separate activation kernel.

Dispatch (GPU): M <= 128 -> ``csrc/kernels/skinny_gemm.hip`` with the (ntw, split-K) plan that the
autotuner measured fastest for this (M, N, K, swiglu) — including "blas" (hipBLASLt via
``F.linear``) as a candidate, so the custom kernel is only used where it wins; M > 128 (prefill)
-> hipBLASLt.  Plans are tuned once per shape OUTSIDE graph capture (``autotune`` is called by the
engine for every decode bucket before capturing); an unseen shape during capture falls back to
a heuristic plan.  CPU tensors -> plain torch.
"""
from __future__ import annotations

import math
import os
from typing import Dict, Iterable, Optional, Tuple

import torch
import torch.nn.functional as F

from . import _native, reference as ref

MAX_M = 256        # custom kernels cover decode buckets up to 256 rows
SKINNY_MAX_M = 128
_SPLITS = (1, 2, 4, 8, 16)
_NTWS = (1, 2, 4)
_MM_NTS = (2, 4)
_MM_SPLITS = (1, 2, 4, 8)
_GEMV_MS = (1, 2, 4, 8)   # csrc/kernels/gemv.hip instantiations (decode buckets below 16)
_GEMV_RS = (1, 2, 4)


class _Planner:
    def __init__(self):
        self.plans: Dict[Tuple[int, int, int, bool], Tuple] = {}
        self.part: Dict[torch.device, torch.Tensor] = {}
        self.counters: Dict[torch.device, torch.Tensor] = {}
        self.timings: Dict[Tuple[int, int, int, bool], Dict[str, float]] = {}

    def workspace(self, dev: torch.device, floats: int, tiles: int):
        p = self.part.get(dev)
        if p is None or p.numel() < floats:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("skinny_gemm workspace growth during graph capture")
            p = torch.empty(max(floats, 1 << 20), dtype=torch.float32, device=dev)
            self.part[dev] = p
        c = self.counters.get(dev)
        if c is None or c.numel() < tiles:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("skinny_gemm counter growth during graph capture")
            c = torch.zeros(max(tiles, 4096), dtype=torch.int32, device=dev)
            self.counters[dev] = c
        return p, c


_P = _Planner()


def _need_mm(M: int, N: int, K: int, nt: int, splits: int) -> Tuple[int, int]:
    bn = 16 * nt
    tiles = (N + bn - 1) // bn
    kchunk = ((K + splits - 1) // splits + 63) // 64 * 64
    S = (K + kchunk - 1) // kchunk
    bm = 64 if M <= 64 else 128 if M <= 128 else 256
    return (S * tiles * bn * bm if S > 1 else 0), tiles


def _need(M: int, N: int, K: int, ntw: int, splits: int, variant: int = 0) -> Tuple[int, int]:
    nc = (16 if variant == 0 else 64) * ntw
    tiles = (N + nc - 1) // nc
    kchunk = ((K + splits - 1) // splits + 31) // 32 * 32
    S = (K + kchunk - 1) // kchunk
    # split-K slabs are laid out with the kernel's row-tile height (MT x 16 rows, MT in 1/2/4/8),
    # not ceil(M/16) x 16: e.g. M = 100 runs the MT = 8 kernel and needs 128-row slabs
    mp = 16 * (1 if M <= 16 else 2 if M <= 32 else 4 if M <= 64 else 8)
    return (S * tiles * nc * mp if S > 1 else 0), tiles


def _heuristic(M: int, N: int, K: int) -> Tuple:
    if M > SKINNY_MAX_M:
        return ("blas",)
    ntw = 1 if M > 64 else 2
    tiles = (N + 16 * ntw - 1) // (16 * ntw)
    splits = max(1, min(16, math.ceil(512 / tiles), K // 256))
    return ("skinny", ntw, splits)


def _run_plan(plan, x, w, swiglu, out):
    if plan[0] == "blas":
        if swiglu:
            x = ref_silu_mul(x)
        return torch.matmul(x, w.t(), out=out) if out is not None else F.linear(x, w)
    ext = _native(x)
    if plan[0] == "gemv":
        y = out if out is not None else torch.empty((x.shape[0], w.shape[0]), dtype=x.dtype, device=x.device)
        ext.gemv(x, w, y, plan[1], swiglu)
        return y
    kind, ntw, splits = plan
    M, N, K = x.shape[0], w.shape[0], w.shape[1]
    y = out if out is not None else torch.empty((M, N), dtype=x.dtype, device=x.device)
    if kind == "mm":
        floats, tiles = _need_mm(M, N, K, ntw, splits)
        part, cnt = _P.workspace(x.device, floats, tiles)
        ext.mm_gemm(x, w, y, ntw, splits, swiglu, part, cnt)
        return y
    variant = 0 if kind == "skinny" else 1
    floats, tiles = _need(M, N, K, ntw, splits, variant)
    part, cnt = _P.workspace(x.device, floats, tiles)
    ext.skinny_gemm(x, w, y, ntw, splits, swiglu, part, cnt, variant)
    return y


def ref_silu_mul(gu):
    from . import silu_mul
    return silu_mul(gu)


def _key(x, w, swiglu):
    return (x.shape[0], w.shape[0], w.shape[1], bool(swiglu))


def linear(x: torch.Tensor, w: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if not x.is_cuda or x.shape[0] > MAX_M or os.environ.get("DLLM_GEMM") == "blas":
        return F.linear(x, w) if out is None else torch.matmul(x, w.t(), out=out)
    plan = _P.plans.get(_key(x, w, False)) or _heuristic(x.shape[0], w.shape[0], w.shape[1])
    return _run_plan(plan, x, w, False, out)


def norm_linear(h: torch.Tensor, residual: torch.Tensor, spare: torch.Tensor, norm_w: torch.Tensor, eps: float,
                w: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """``linear(rmsnorm(h + residual) * norm_w, w)`` and the updated residual stream.

    Where the tuned plan for this shape is the GEMV (batch <= 8), one launch does both
    (csrc/kernels/gemv.hip NORM): the new residual goes to ``spare`` and is returned; otherwise
    the norm kernel updates ``residual`` in place and it is returned.  Callers keep whichever
    buffer comes back as the residual and the other one as the next spare.

    Opt-in (DLLM_FUSED_NORM=1): measured SLOWER on MI355X at batch 1 (0.954 vs 0.889 ms per
    TinyLlama decode step, profiles/r1_small_batch_decode.md) -- every GEMV workgroup redoes the
    norm's reduction and two extra L2 round trips sit before its first FMA, which costs more
    than the separate 4.5 us norm launch it removes."""
    M, N, K = h.shape[0], w.shape[0], w.shape[1]
    if h.is_cuda and M <= MAX_M and os.environ.get("DLLM_GEMM") != "blas" \
            and os.environ.get("DLLM_FUSED_NORM", "0") == "1":
        plan = _P.plans.get((M, N, K, False))
        if plan is not None and plan[0] == "gemv" and h.is_contiguous() and M * K * 2 <= 64 * 1024:
            y = torch.empty((M, N), dtype=h.dtype, device=h.device)
            _native(h).gemv_norm(h, residual, spare, norm_w, float(eps), w, y, plan[1])
            return y, spare
    from . import rms_norm
    x = rms_norm(h, norm_w, eps, residual=residual)
    return linear(x, w), residual


def linear_swiglu(gu: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """``silu(gate) * up @ w.T`` with gu = [gate | up] of width 2K."""
    if not gu.is_cuda:
        return F.linear(ref.silu_mul(gu), w)
    if gu.shape[0] > MAX_M or os.environ.get("DLLM_GEMM") == "blas":
        from . import silu_mul
        return F.linear(silu_mul(gu), w)
    plan = _P.plans.get(_key(gu, w, True)) or _heuristic(gu.shape[0], w.shape[0], w.shape[1])
    return _run_plan(plan, gu, w, True, None)


def _time(fn, iters=24) -> float:
    """GPU time per call of fn(i) in us, measured as a hipGraph replay of ``iters`` calls (the
    decode step is a graph replay too, so host launch cost is excluded exactly as in serving).
    Callers rotate operands over i so weights come from HBM, not the 256 MiB Infinity Cache
    (a decode step streams the whole model: its weights are cold)."""
    fn(0)  # eager warm-up: allocates workspaces / initialises libraries outside capture
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


def autotune(shapes: Iterable[Tuple[int, int, bool]], ms: Iterable[int], device, verbose: bool = False) -> None:
    """Measure every candidate plan for each (M, N, K, swiglu) and keep the fastest."""
    dev = torch.device(device)
    if dev.type != "cuda" or os.environ.get("DLLM_GEMM") == "blas":
        return
    cache = os.environ.get("DLLM_GEMM_PLANS")  # JSON plan cache: re-use a previous run's choices
    if cache and os.path.exists(cache):
        import json
        with open(cache) as f:
            for k, v in json.load(f).items():
                M, N, K, sw = k.split(",")
                _P.plans[(int(M), int(N), int(K), sw == "1")] = tuple(v)
    shapes = list(shapes)
    _autotune(shapes, list(ms), dev, verbose)
    if cache:
        import json
        with open(cache, "w") as f:
            json.dump({f"{M},{N},{K},{int(sw)}": list(v) for (M, N, K, sw), v in _P.plans.items()}, f)


def _autotune(shapes, ms, dev, verbose: bool) -> None:
    for (N, K, sw) in shapes:
        copies = max(2, min(64, math.ceil((768 << 20) / (N * K * 2))))
        ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(copies)]
        for M in ms:
            if M > MAX_M:
                continue
            key = (M, N, K, sw)
            if key in _P.plans:
                continue
            x = torch.randn(M, 2 * K if sw else K, device=dev).to(torch.bfloat16)
            cands = [("blas",)]
            if M > 16 and K % 64 == 0 and N % 8 == 0 and os.environ.get("DLLM_GEMM_NO_MM") != "1":
                for nt in _MM_NTS:
                    for s in _MM_SPLITS:
                        if s > 1 and K // s < 256:
                            continue
                        floats, _ = _need_mm(M, N, K, nt, s)
                        if floats * 4 > 256 << 20:
                            continue
                        cands.append(("mm", nt, s))
            if M in _GEMV_MS and K % 8 == 0 and M * K * 2 <= 64 * 1024 and os.environ.get("DLLM_GEMM_NO_GEMV") != "1":
                cands.extend(("gemv", r) for r in _GEMV_RS)
            for kind, ntws in ((("skinny", _NTWS), ("lds", (1, 2))) if M <= SKINNY_MAX_M else ()):
                for ntw in ntws:
                    if M > 64 and (ntw == 4 or (kind == "lds" and ntw == 2)):
                        continue
                    for s in _SPLITS:
                        if s > 1 and K // s < 128:
                            continue
                        floats, _ = _need(M, N, K, ntw, s, 0 if kind == "skinny" else 1)
                        if floats * 4 > 256 << 20:
                            continue
                        cands.append((kind, ntw, s))
            res = {}
            for c in cands:
                res[c] = _time(lambda i: _run_plan(c, x, ws[i % copies], sw, None))
            best = min(res, key=res.get)
            _P.plans[key] = best
            _P.timings[key] = {str(c): round(t, 2) for c, t in res.items()}
            if verbose:
                bk = {k: min((c for c in res if c[0] == k), key=res.get, default=None)
                      for k in ("gemv", "skinny", "lds", "mm")}
                extra = " ".join(f"{k}={c[1:]}:{res[c]:.1f}us" for k, c in bk.items() if c)
                print(f"gemm M={M} N={N} K={K} swiglu={sw}: best={best} {res[best]:.1f}us "
                      f"({N * K * 2 / res[best] / 1e3:.0f} GB/s; blas {res[('blas',)]:.1f}us; {extra})", flush=True)
        del ws


def plans() -> Dict:
    return {str(k): v for k, v in _P.plans.items()}
