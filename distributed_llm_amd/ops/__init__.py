"""Op library: HIP/CDNA4 kernels (``_hip_kernels`` extension) with plain-PyTorch references.

Dispatch rule: GPU tensors ALWAYS run the HIP kernel.  If the extension is missing on a GPU
box the call raises (``NativeOpsMissing``) — there is no silent eager fallback
(set ``DLLM_ALLOW_TORCH_FALLBACK=1`` only for debugging).  CPU tensors run the torch
reference implementation (``ops.reference``), which is also what the kernel numerics tests
compare against.

KV-cache layout (per layer):  K [num_blocks, nkv, 16, d],  V [num_blocks, nkv, d, 16]
(V transposed per block — see csrc/kernels/attention.hip).
"""
from __future__ import annotations

import math
import os
import struct
from typing import List, Optional, Tuple

import numpy as np
import torch

from . import reference as ref

BLOCK_SIZE = 16

_ext = None
_ext_err: Optional[BaseException] = None


class NativeOpsMissing(RuntimeError):
    pass


def _load():
    global _ext, _ext_err
    if _ext is not None or _ext_err is not None:
        return _ext
    try:
        from . import _hip_kernels  # type: ignore
        _ext = _hip_kernels
    except BaseException as e:  # ImportError or a loader error
        _ext_err = e
    return _ext


def native_available() -> bool:
    return _load() is not None


def _native(t: torch.Tensor):
    """Return the extension for a GPU tensor, None for CPU tensors; raise if missing on GPU."""
    if not t.is_cuda:
        return None
    ext = _load()
    if ext is None:
        if os.environ.get("DLLM_ALLOW_TORCH_FALLBACK") == "1":
            return None
        raise NativeOpsMissing(
            f"HIP kernel extension not built/loadable ({_ext_err}); run "
            "`python -m distributed_llm_amd._build` (gfx950)")
    return ext


# ----------------------------------------------------------------------------- norms

def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float, residual: Optional[torch.Tensor] = None,
             out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = rmsnorm(x + residual) * w;  ``residual`` is updated in place to ``x + residual``."""
    ext = _native(x)
    if ext is None:
        return ref.rms_norm(x, w, eps, residual)
    y = out if out is not None else torch.empty_like(x)
    ext.norm(x, residual, w, None, y, eps, False)
    return y


def layer_norm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float,
               residual: Optional[torch.Tensor] = None) -> torch.Tensor:
    ext = _native(x)
    if ext is None:
        return ref.layer_norm(x, w, b, eps, residual)
    y = torch.empty_like(x)
    ext.norm(x, residual, w, b, y, eps, True)
    return y


# ----------------------------------------------------------------------------- rope + kv

def rope_cos_sin(max_pos: int, d: int, theta: float, device=None, scaling: Optional[dict] = None) -> torch.Tensor:
    """Host-precomputed [max_pos, d] f32 table: cos in [:d/2], sin in [d/2:]."""
    inv = 1.0 / (theta ** (torch.arange(0, d, 2, dtype=torch.float64) / d))
    if scaling and scaling.get("rope_type") == "llama3":
        inv = ref.llama3_scale_inv_freq(inv, scaling)
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv)
    return torch.cat([f.cos(), f.sin()], dim=1).float().to(device)


def rope_and_cache(qkv: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor, slots: torch.Tensor,
                   k_cache: torch.Tensor, v_cache: torch.Tensor, nq: int, nkv: int, d: int,
                   q_out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Rotate q/k, write k and v into the paged caches, return q as [T, nq, d]."""
    ext = _native(qkv)
    if ext is None:
        return ref.rope_and_cache(qkv, positions, cos_sin, slots, k_cache, v_cache, nq, nkv, d)
    T = qkv.shape[0]
    q = q_out if q_out is not None else torch.empty((T, nq, d), dtype=qkv.dtype, device=qkv.device)
    ext.rope_kv(qkv, positions, cos_sin, slots, q, k_cache, v_cache, nq, nkv, d)
    return q


def kv_write(k: torch.Tensor, v: torch.Tensor, slots: torch.Tensor, k_cache: torch.Tensor,
             v_cache: torch.Tensor) -> None:
    ext = _native(k)
    if ext is None:
        return ref.kv_write(k, v, slots, k_cache, v_cache)
    ext.kv_write(k.contiguous(), v.contiguous(), slots, k_cache, v_cache)


# ----------------------------------------------------------------------------- attention

def build_tiles(q_lens, group: int) -> Tuple[list, list]:
    """Host tile table: each 16-row tile covers 16/group tokens of one sequence."""
    tpt = 16 // group
    ts, tt = [], []
    for s, n in enumerate(q_lens):
        for t0 in range(0, int(n), tpt):
            ts.append(s)
            tt.append(t0)
    return ts, tt


def paged_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, block_tables: torch.Tensor,
                    seq_qstart: torch.Tensor, seq_qlen: torch.Tensor, seq_ctx: torch.Tensor,
                    tile_seq: torch.Tensor, tile_tok0: torch.Tensor, scale: Optional[float] = None,
                    causal: bool = True, splits: int = 1, out: Optional[torch.Tensor] = None,
                    workspace: Optional[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]] = None,
                    split_len: Optional[torch.Tensor] = None, xcd_remap: bool = False,
                    items: Optional[torch.Tensor] = None, grid_items: int = 0,
                    v_new: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Paged attention over new query tokens ``q [T, nq, d]`` (see csrc/kernels/attention.hip).

    ``v_new`` (decode, one query token per sequence): the new tokens' V row-major [T, nkv * d],
    NOT yet in the V^T cache (``gemm.qkv_rope_cache(v_new=...)``); the kernel writes each
    sequence's newest V into the cache and uses it (CPU: the reference writes it first).  GPU:
    head_dim 64 with the work list only (the patch would cost d = 96 / 128 a wave per SIMD).

    ``splits`` is the split-K grid depth; with ``split_len`` (int32 device scalar, keys per split)
    each tile uses only ceil(its keys / split_len) of them (dynamic, balanced split-K).
    ``xcd_remap``: XCD-contiguous block order, for prefill (K/V re-read by a sequence's tiles hits
    one XCD's L2).
    ``items`` (decode): a work list from :func:`decode_work_items`; a fixed grid of ``grid_items``
    workgroups walks it (``splits`` is then the workspace split stride)."""
    d = q.shape[-1]
    scale = (1.0 / math.sqrt(d)) if scale is None else scale
    ext = _native(q)
    if ext is None:
        if v_new is not None:   # the newest token of each sequence: V into the V^T cache first
            ref.write_newest_v(v_new, v_cache, block_tables, seq_qstart, seq_ctx)
        return ref.paged_attention(q, k_cache, v_cache, block_tables, seq_qstart, seq_qlen, seq_ctx, scale, causal)
    o = out if out is not None else torch.empty_like(q)
    po = pml = cnt = None
    if splits > 1:
        if workspace is None:
            nt, nkv = tile_seq.numel(), k_cache.shape[1]
            po = torch.empty(nt * nkv * splits * 16 * d, dtype=torch.float32, device=q.device)
            pml = torch.empty(nt * nkv * splits * 16 * 2, dtype=torch.float32, device=q.device)
            cnt = torch.zeros(nt * nkv, dtype=torch.int32, device=q.device)
        else:
            po, pml, cnt = workspace
    ext.paged_attention(q, k_cache, v_cache, block_tables, seq_qstart, seq_qlen, seq_ctx, tile_seq, tile_tok0, o,
                        po, pml, cnt, splits, causal, scale, split_len if splits > 1 and items is None else None,
                        xcd_remap, items, int(grid_items), v_new)
    return o


FLASH_ROWS = 256


FLASH_CK, FLASH_STAGES = 64, 3   # csrc/kernels/flash_prefill.hip: keys per chunk, K/V ring depth


def flash_lds_bytes(d: int, max_blocks: int) -> int:
    """Dynamic LDS of the flash prefill kernel's plain loop (the launcher's formula): the K/V ring
    plus the tile's whole block-table row, staged once per workgroup (no re-staging window)."""
    return FLASH_STAGES * (2 * FLASH_CK * d * 2) + (max_blocks * 4 + 15) // 16 * 16


def flash_supported(d: int, group: int, max_blocks: int) -> bool:
    """The flash kernel stages a tile's ENTIRE block-table row in LDS, sized at launch: it runs any
    context whose table fits next to the 3-stage K/V ring in the 160 KB: 16,384 blocks = 262K keys at
    d = 128, 360K at d = 96, 458K at d = 64 (the pipelined d = 128 form needs 48 KB more and falls
    back to the plain loop on its own).  Longer contexts are served by the slower paged kernel
    (``paged_attention``) instead of failing at launch (dllm_flash_prefill returns -3)."""
    return d in (64, 96, 128) and FLASH_ROWS % group == 0 and max_blocks >= 1 and \
        flash_lds_bytes(d, max_blocks) <= 160 * 1024 and os.environ.get("DLLM_FLASH_PREFILL", "1") == "1"


def flash_tiles(q_lens, group: int) -> Tuple[list, list]:
    """Host tile table of the flash prefill kernel: 256 / group query tokens per tile."""
    tpt = FLASH_ROWS // group
    ts, tt = [], []
    for s, n in enumerate(q_lens):
        for t0 in range(0, int(n), tpt):
            ts.append(s)
            tt.append(t0)
    return ts, tt


def flash_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, block_tables: torch.Tensor,
                    seq_qstart: torch.Tensor, seq_qlen: torch.Tensor, seq_ctx: torch.Tensor, tile_seq: torch.Tensor,
                    tile_tok0: torch.Tensor, scale: Optional[float] = None, causal: bool = True,
                    out: Optional[torch.Tensor] = None, max_ctx: int = 0) -> torch.Tensor:
    """Flash-style prefill over the paged cache (csrc/kernels/flash_prefill.hip); tiles from
    :func:`flash_tiles`.  Same contract as :func:`paged_attention` (CPU: the same reference).
    ``max_ctx`` (host-known longest context, 0 = unknown) enables split-KV for small grids."""
    d = q.shape[-1]
    scale = (1.0 / math.sqrt(d)) if scale is None else scale
    ext = _native(q)
    if ext is None:
        return ref.paged_attention(q, k_cache, v_cache, block_tables, seq_qstart, seq_qlen, seq_ctx, scale, causal)
    o = out if out is not None else torch.empty_like(q)
    units = int(tile_seq.numel()) * int(k_cache.shape[1])
    sp = flash_splits(units, max_ctx)
    # the kernel addresses its split partials through 32-bit buffer descriptors: keep the O
    # partials under 2 GiB (a forced DLLM_FLASH_SPLITS on a long prompt could exceed it: ADVICE r4)
    while sp > 1 and units * sp * FLASH_ROWS * d * 4 >= (1 << 31):
        sp -= 1
    if sp > 1:
        po, pml, cnt = _flash_workspace(q.device, units * sp * FLASH_ROWS * d, units * sp * FLASH_ROWS * 4, units)
        ext.flash_prefill(q, k_cache, v_cache, block_tables, seq_qstart, seq_qlen, seq_ctx, tile_seq, tile_tok0, o,
                          causal, scale, sp, po, pml, cnt)
    else:
        ext.flash_prefill(q, k_cache, v_cache, block_tables, seq_qstart, seq_qlen, seq_ctx, tile_seq, tile_tok0, o,
                          causal, scale)
    return o


# Split-KV for flash grids that leave CUs idle: each (tile, kv head) unit's key chunks are dealt to
# `splits` workgroups and the last one combines their partials.  Measured (profiles/r4_flash_split.md):
# the partial write + ticket + combine costs more than it saves on a cold 1K prompt (short key chains:
# 50 vs 35 us), so it is only chosen for a small grid over LONG contexts (a few new tokens behind a
# long cached history: one unit walks thousands of keys).  DLLM_FLASH_SPLITS=N forces N (1 = off).
FLASH_SPLIT_TARGET = 512
FLASH_SPLIT_MIN_CTX = 4096


def flash_splits(units: int, max_ctx: int = 0) -> int:
    e = os.environ.get("DLLM_FLASH_SPLITS")
    if e is not None:
        return max(1, min(16, int(e)))
    if units <= 0 or units >= FLASH_SPLIT_TARGET // 2 or max_ctx < FLASH_SPLIT_MIN_CTX:
        return 1
    return max(1, min(8, -(-FLASH_SPLIT_TARGET // units), max_ctx // 2048))


def _flash_workspace(dev, n_o: int, n_ml: int, n_cnt: int):
    """Split-KV workspace of ONE launch (partials and tickets; the launcher zeroes the tickets),
    from the caching allocator on the current stream: two engines prefilling on one device
    (co-located tiers, separate step loops and streams) never share partials or tickets."""
    return (torch.empty(n_o, dtype=torch.float32, device=dev), torch.empty(n_ml, dtype=torch.float32, device=dev),
            torch.empty(n_cnt, dtype=torch.int32, device=dev))


def decode_work_items(ctx, nkv: int, max_splits: int, target_items: int, min_chunk: int = 256,
                      out: Optional[np.ndarray] = None, seq=None, qstart=None) -> np.ndarray:
    """Work list for persistent decode attention (one query token per tile, tiles in ``ctx`` order).

    Every (tile, kv head) is cut into ``ceil(ctx / chunk)`` splits (at most ``max_splits``) with
    ``chunk`` sized so the batch yields about ``target_items`` units; units are emitted tile by
    tile, so with tiles sorted longest context first the list runs from the largest units to the
    smallest (round-robin over the grid then approximates longest-processing-time scheduling).
    Returns int32 ``[1 + 2n]``: ``n``, then ``(tile | kvh << 16, split | nsplit << 8)`` pairs.

    With ``seq`` / ``qstart`` (per tile: block-table row and query row) the list is the extended
    form ``[4 + 4n]``: ``-n``, three pad words, then 16-byte units ``(tile | kvh << 16,
    split | nsplit << 8, seq | qstart << 16, ctx)``, so the kernel reads a unit's sequence
    metadata with the unit instead of through two more dependent loads.
    """
    ctx = np.asarray(ctx, dtype=np.int64)
    B = ctx.shape[0]
    total = int(ctx.sum())
    chunk = max(min_chunk, -(-total * nkv // max(1, target_items)))
    chunk = (chunk + 31) & ~31
    ns = np.clip(-(-ctx // chunk), 1, max_splits)
    rep = ns * nkv
    n = int(rep.sum())
    starts = np.cumsum(rep) - rep
    j = np.arange(n, dtype=np.int64) - np.repeat(starts, rep)
    ns_r = np.repeat(ns, rep)
    tile = np.repeat(np.arange(B, dtype=np.int64), rep)
    ext = seq is not None
    head, width = (4, 4) if ext else (1, 2)
    buf = out if out is not None else np.empty(head + width * n, dtype=np.int32)
    buf[0] = -n if ext else n
    w = buf[head:head + width * n].reshape(n, width)
    w[:, 0] = tile | ((j // ns_r) << 16)
    w[:, 1] = (j % ns_r) | (ns_r << 8)
    if ext:
        buf[1:4] = 0
        seq = np.asarray(seq, dtype=np.int64)
        qstart = np.asarray(qstart, dtype=np.int64)
        w[:, 2] = np.repeat(seq | (qstart << 16), rep)
        w[:, 3] = np.repeat(ctx, rep)
    return buf


def work_items_len(items: np.ndarray) -> int:
    """Number of int32 words of a :func:`decode_work_items` list (either form)."""
    n = int(items[0])
    return 4 + 4 * (-n) if n < 0 else 1 + 2 * n


# ----------------------------------------------------------------------------- activations

def silu_mul(gu: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    ext = _native(gu)
    if ext is None:
        return ref.silu_mul(gu)
    T, I2 = gu.shape
    o = out if out is not None else torch.empty((T, I2 // 2), dtype=gu.dtype, device=gu.device)
    ext.silu_mul(gu, o)
    return o


def embedding(ids: torch.Tensor, table: torch.Tensor, lo: int = 0,
              ssq_out: Optional[torch.Tensor] = None,
              scatter: Optional[Tuple[torch.Tensor, torch.Tensor]] = None) -> torch.Tensor:
    """Row gather ``table[ids - lo]`` -> [T, H]; ids outside ``[lo, lo + rows)`` give zero rows
    (vocab-parallel shard of a TP rank: the all-reduce then sums the owners' rows).  ``ssq_out``
    (f32, >= T): also each row's sum of squares, in the same launch.  ``scatter`` = (dst, buf):
    also apply ``scatter_pairs(dst, buf)`` (a decode step's block-table updates) in the same launch."""
    ext = _native(table)
    if ext is None:
        if scatter is not None:
            scatter_pairs(*scatter)
        out = ref.embedding(ids, table, lo)
        if ssq_out is not None:
            ssq_out[:out.shape[0]] = (out.float() ** 2).sum(1)
        return out
    ids = ids.reshape(-1).to(torch.int32).contiguous()
    out = torch.empty((ids.numel(), table.shape[1]), dtype=table.dtype, device=table.device)
    if scatter is None:
        ext.embed(ids, table, out, int(lo), ssq_out)
    else:
        ext.embed(ids, table, out, int(lo), ssq_out, scatter[0], scatter[1])
    return out


def gelu(x: torch.Tensor) -> torch.Tensor:
    ext = _native(x)
    if ext is None:
        return ref.gelu(x)
    x = x.contiguous()
    y = torch.empty_like(x)
    ext.gelu(x, y)
    return y


def encoder_attention(qkv: torch.Tensor, lens: torch.Tensor, B: int, S: int, nh: int, d: int,
                      scale: Optional[float] = None) -> torch.Tensor:
    """Bidirectional (encoder) attention over a padded batch, qkv [B*S, 3 nh d] -> [B*S, nh d];
    keys at positions >= lens[b] are masked (csrc/kernels/encoder.hip)."""
    scale = (1.0 / math.sqrt(d)) if scale is None else scale
    ext = _native(qkv)
    if ext is None:
        return ref.encoder_attention(qkv, lens, B, S, nh, d, scale)
    out = torch.empty((B * S, nh * d), dtype=qkv.dtype, device=qkv.device)
    ext.encoder_attention(qkv.contiguous(), lens.to(torch.int32).contiguous(), out, B, S, nh, d, float(scale))
    return out


def embed_ln(ids: torch.Tensor, word: torch.Tensor, pos: torch.Tensor, type0: torch.Tensor, w: torch.Tensor,
             b: torch.Tensor, S: int, eps: float) -> torch.Tensor:
    """BERT embeddings: LayerNorm(word[ids] + pos[t % S] + type0) for ids [B, S] -> [B*S, H]."""
    ext = _native(word)
    if ext is None:
        return ref.embed_ln(ids, word, pos, type0, w, b, S, eps)
    ids = ids.reshape(-1).to(torch.int32).contiguous()
    out = torch.empty((ids.numel(), word.shape[1]), dtype=word.dtype, device=word.device)
    ext.embed_ln(ids, word, pos, type0, w, b, out, int(S), float(eps))
    return out


def mean_pool_l2(x: torch.Tensor, lens: torch.Tensor) -> torch.Tensor:
    ext = _native(x)
    if ext is None:
        return ref.mean_pool_l2(x, lens)
    out = torch.empty((x.shape[0], x.shape[2]), dtype=torch.float32, device=x.device)
    ext.mean_pool_l2(x.contiguous(), lens.to(torch.int32).contiguous(), out)
    return out


def moe_gate(logits: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
    ext = _native(logits)
    if ext is None:
        return ref.moe_gate(logits, k)
    T = logits.shape[0]
    ids = torch.empty((T, k), dtype=torch.int32, device=logits.device)
    w = torch.empty((T, k), dtype=torch.float32, device=logits.device)
    ext.moe_gate(logits.float().contiguous(), k, ids, w)
    return ids, w


def moe_router(x: torch.Tensor, wg: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Router projection + top-k in one kernel (csrc/kernels/elementwise.hip moe_router_kernel):
    fp32 logits x . wg^T with a per-token fixed reduction order, so routing is batch-invariant (a
    padded graph batch picks the same experts as the eager batch; a vendor GEMM's split varies
    with M).  x [T, H] bf16, wg [E, H] bf16 -> ids [T, k] int32, renormalised weights [T, k] f32."""
    ext = _native(x)
    if ext is None or x.shape[1] > 8192 or x.shape[1] % 8 or x.stride(0) % 8 or x.data_ptr() % 16 or wg.data_ptr() % 16:
        return moe_gate(torch.nn.functional.linear(x.float(), wg.float()), k)
    T = x.shape[0]
    ids = torch.empty((T, k), dtype=torch.int32, device=x.device)
    w = torch.empty((T, k), dtype=torch.float32, device=x.device)
    ext.moe_router(x if x.stride(1) == 1 else x.contiguous(), wg.contiguous(), k, ids, w)
    return ids, w


def moe_ffn(x: torch.Tensor, ids: torch.Tensor, wts: torch.Tensor, w13: torch.Tensor,
            w2: torch.Tensor) -> torch.Tensor:
    """Top-k expert FFN (csrc/kernels/moe.hip): device-side routing + grouped MFMA GEMMs with the
    SwiGLU in the first GEMM's epilogue; graph-capturable.  x [T, H], ids [T, k] int32,
    wts [T, k] f32, w13 [E, 2I, H], w2 [E, H, I] -> [T, H]."""
    ext = _native(x)
    if ext is None:
        return ref.moe_ffn(x, ids, wts, w13, w2)
    out = torch.empty((x.shape[0], x.shape[1]), dtype=x.dtype, device=x.device)
    ext.moe_ffn(x, ids.to(torch.int32).contiguous(), wts.float().contiguous(), w13, w2, out)
    return out


MOE_PLANS = {  # (bm, bn13, stages13, ks13, nw13, bn2, stages2, ks2, nw2) by routed-pair count
    # measured at Mixtral shapes (profiles/r2_moe_microbench.md)
    "decode": (64, 128, 3, 1, 4, 64, 6, 1, 4),        # P <= 128: weight streaming, 64-row tiles, 6-deep ring for
                                                      # the long-K down projection
    "mid": (128, 128, 4, 1, 8, 128, 4, 1, 8),         # P <= 1024
    "prefill": (256, 256, 2, 1, 8, 128, 3, 1, 8),     # large P: 256x256 tiles (weight reuse)
}


def moe_plan(pairs: int) -> Tuple[int, ...]:
    return MOE_PLANS["decode" if pairs <= 128 else "mid" if pairs <= 1024 else "prefill"]


def moe_ffn_tg(x: torch.Tensor, ids: torch.Tensor, wts: torch.Tensor, w13i: torch.Tensor, w2: torch.Tensor,
               plan: Optional[Tuple[int, ...]] = None) -> torch.Tensor:
    """Top-k expert FFN on the grouped LDS-tiled MFMA GEMM (csrc/kernels/moe.hip moe_ffn_tg):
    ``w13i`` [E, 2I, H] with gate/up rows interleaved in 16-row groups (models.llama.gate_up_order),
    w2 [E, H, I].  Routing, both GEMMs and the weighted combine stay on the device."""
    ext = _native(x)
    if ext is None:
        from ..models.llama import gate_up_order
        w13 = torch.empty_like(w13i)
        w13[:, gate_up_order(w13i.shape[1] // 2)] = w13i
        return ref.moe_ffn(x, ids, wts, w13, w2)
    out = torch.empty((x.shape[0], x.shape[1]), dtype=x.dtype, device=x.device)
    if plan is None:
        plan = moe_plan(x.shape[0] * ids.shape[1])
    ext.moe_ffn_tg(x, ids.to(torch.int32).contiguous(), wts.float().contiguous(), w13i, w2, out, list(plan))
    return out


# ----------------------------------------------------------------------------- sampling

def argmax(logits: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    ext = _native(logits)
    if ext is None:
        return torch.argmax(logits.float(), dim=-1).to(torch.int32)
    o = out if out is not None else torch.empty(logits.shape[0], dtype=torch.int32, device=logits.device)
    ext.argmax(logits, o)
    return o


def sample_top_p(cand_vals: torch.Tensor, cand_idx: torch.Tensor, temperature: torch.Tensor, top_p: torch.Tensor,
                 uniform: torch.Tensor) -> torch.Tensor:
    """Nucleus sampling over sorted top-k candidates (values descending)."""
    ext = _native(cand_vals)
    if ext is None:
        return ref.sample_top_p(cand_vals, cand_idx, temperature, top_p, uniform)
    o = torch.empty(cand_vals.shape[0], dtype=torch.int32, device=cand_vals.device)
    ext.sample_topp(cand_vals.float().contiguous(), cand_idx.contiguous(), temperature.float().contiguous(),
                    top_p.float().contiguous(), uniform.float().contiguous(), o)
    return o


def sample_rows(logits: torch.Tensor, temperature: torch.Tensor, top_p: torch.Tensor, top_k: torch.Tensor,
                seed: torch.Tensor, out: Optional[torch.Tensor] = None, shards: Optional[int] = None) -> torch.Tensor:
    """One-launch sampler over bf16 logits [B, V] (csrc/kernels/sampling.hip sample_rows_kernel):
    per row, temperature <= 0 -> arg-max, else exact top-k (top_k <= 0 -> 256 candidates),
    temperature, top-p and an inverse-CDF draw with u = hash(seed, row).  All parameters are
    device tensors (f32 / int32, ``seed`` an int32 scalar), so the call is graph-capturable.
    Small batches of large-vocab rows run sample_split_kernel instead (the row's vocab on up to 8
    workgroups, same tokens; ``sample_split_shards``); ``shards`` forces a shard count (1: never)."""
    ext = _native(logits)
    if ext is None:
        r = ref.sample_rows(logits, temperature.cpu(), top_p.cpu(), top_k.cpu(), int(seed.reshape(-1)[0]))
        if out is not None:
            out[:r.numel()].copy_(r)
            return out
        return r
    o = out if out is not None else torch.empty(logits.shape[0], dtype=torch.int32, device=logits.device)
    B, V = logits.shape
    P = sample_split_shards(B, V) if shards is None else max(1, min(8, int(shards)))
    if P > 1:
        # small batch: P vocab shards per row on P workgroups, merged by the row's last arriver
        # (sample_split_kernel); the ranked lists go through the owner's split-K workspace
        from . import gemm as _gemm
        part, counters = _gemm._P.workspace(logits.device, B * P * SAMPLE_SPLIT_KMAX * 2, B)
        ext.sample_split(logits, temperature, top_p, top_k, seed, part, counters, o, P)
    else:
        ext.sample_rows(logits, temperature, top_p, top_k, seed, o)
    return o


SAMPLE_SPLIT_KMAX = 256      # csrc/kernels/sampling.hip SR_KMAX (per-shard list capacity)
SAMPLE_SPLIT_MAX_B = int(os.environ.get("DLLM_SAMPLE_SPLIT_MAX_B", "8"))
SAMPLE_SPLIT_SHARD = 4096    # logits per shard at least (smaller shards: merge cost > load time)
SAMPLE_SPLIT_MIN_V = 65536   # below, one workgroup per row is as fast for sampled rows


def sample_split_shards(B: int, V: int) -> int:
    """Vocab shards per row for ``sample_rows``: 1 (one workgroup per row) unless the batch is
    small (<= ``DLLM_SAMPLE_SPLIT_MAX_B``, 0 disables) and the vocab large (>= 64K), then up to 8
    shards of >= 4096 logits.  Batch 1, top-k 40 (profiles/r4_sampler.md): 128K vocab 52 -> 38 us,
    greedy 26 -> 9 us; at 32K the split only helps greedy rows (9.5 -> 5.9 us) and costs sampled
    ones 3 us, so 32K rows stay on one workgroup."""
    if B > SAMPLE_SPLIT_MAX_B or V < SAMPLE_SPLIT_MIN_V:
        return 1
    return max(1, min(8, V // SAMPLE_SPLIT_SHARD))


TP_KC = 256   # candidates per vocab shard (csrc/kernels/sampling.hip TP_KC)


def tp_candidates(logits: torch.Tensor, start: int) -> torch.Tensor:
    """A vocab shard's ranked top-``TP_KC`` candidates per row as int32 pairs [S, TP_KC, 2] =
    (value as f32 bits, global id = local index + ``start``), order value desc / id asc; rows with
    fewer candidates are padded with (-inf, INT32_MAX).  One launch (tp_cands_kernel)."""
    ext = _native(logits)
    if ext is None:
        return ref.tp_candidates(logits, start, TP_KC)
    cand = torch.empty((logits.shape[0], TP_KC, 2), dtype=torch.int32, device=logits.device)
    ext.tp_cands(logits, int(start), cand)
    return cand


def tp_sample(cands: torch.Tensor, temperature: torch.Tensor, top_p: torch.Tensor, top_k: torch.Tensor,
              seed: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Token per row from the all-gathered shard candidates ``cands`` [tp, S, TP_KC, 2]: merge the
    tp ranked lists and draw exactly as ``sample_rows`` would on the unsharded row (greedy ->
    best id; else top-k, temperature, top-p, u = hash(seed, row)).  One launch (tp_sample_kernel)."""
    S = cands.shape[1]
    o = out if out is not None else torch.empty(S, dtype=torch.int32, device=cands.device)
    ext = _native(cands)
    if ext is None:
        r = ref.tp_sample(cands, temperature.cpu(), top_p.cpu(), top_k.cpu(), int(seed.reshape(-1)[0]))
        o[:S].copy_(r)
        return o
    ext.tp_sample(cands.contiguous(), temperature, top_p, top_k, seed, o)
    return o


# ----------------------------------------------------------------------------- router scorers

def cosine_scores(q: torch.Tensor, c: torch.Tensor) -> torch.Tensor:
    ext = _native(q)
    if ext is None:
        return ref.cosine_scores(q, c)
    q = q.float().contiguous()
    c = c.float().contiguous()
    s = torch.empty((q.shape[0], c.shape[0]), dtype=torch.float32, device=q.device)
    ext.cosine_scores(q, c, s)
    return s


def _unpack_key(key: int) -> Tuple[int, float]:
    key &= 0xFFFFFFFFFFFFFFFF
    if key == 0:
        return -1, 0.0
    row = 0xFFFFFFFF - (key & 0xFFFFFFFF)
    bits = key >> 32
    bits = (bits & 0x7FFFFFFF) if (bits & 0x80000000) else (~bits & 0xFFFFFFFF)
    return int(row), float(struct.unpack("<f", struct.pack("<I", bits))[0])


CACHE_SCAN_MAX_Q = 128   # queries per cache_scan launch (csrc/kernels/cosine.hip CQ)
CACHE_WRITE_MAX = 64     # row writes per cache_write launch (CW)


def cache_scan(queries: List[torch.Tensor], cids: List[int], table: torch.Tensor, ctx: torch.Tensor, n_rows: int,
               thr: float) -> List[Tuple[int, float]]:
    """Semantic-cache lookups of a routing batch: for each query (an f32 [d] vector) the row of
    ``table[:n_rows]`` whose context id equals the query's with the highest cosine >= thr, as
    (row, sim), or (-1, 0.0).  One launch per 128 queries and ONE host read-back for the batch;
    only rows of the batch's contexts are read (csrc/kernels/cosine.hip cache_scan_kernel)."""
    if not queries:
        return []
    ext = _native(table)
    if ext is None:
        return ref.cache_scan(queries, cids, table, ctx, n_rows, thr)
    qs = [q if (q.dtype == torch.float32 and q.is_contiguous() and q.data_ptr() % 16 == 0) else
          q.float().contiguous() for q in queries]
    best = torch.empty(len(qs), dtype=torch.int64, device=table.device)
    for i in range(0, len(qs), CACHE_SCAN_MAX_Q):
        part = qs[i:i + CACHE_SCAN_MAX_Q]
        ext.cache_scan([q.data_ptr() for q in part], [int(c) for c in cids[i:i + CACHE_SCAN_MAX_Q]], table, ctx,
                       int(n_rows), float(thr), best[i:])
    return [_unpack_key(k) for k in best.tolist()]


def cache_write(writes: List[Tuple[int, Optional[torch.Tensor], int]], table: torch.Tensor, ctx: torch.Tensor) -> None:
    """Apply deferred routing-cache table writes (slot, f32 [d] vector or None, context id) in
    launches of 64: row ``slot`` <- the vector (None: keep the row's bytes), ``ctx[slot]`` <- id
    (-1 removes the row from every lookup).  Slots must be unique within ``writes``."""
    if not writes:
        return
    ext = _native(table)
    if ext is None:
        for slot, v, cid in writes:
            if v is not None:
                table[slot].copy_(v.reshape(-1))
            ctx[slot] = cid
        return
    keep = []
    for i in range(0, len(writes), CACHE_WRITE_MAX):
        part = writes[i:i + CACHE_WRITE_MAX]
        srcs = []
        for _, v, _ in part:
            if v is None:
                srcs.append(0)
                continue
            if not (v.dtype == torch.float32 and v.is_contiguous() and v.data_ptr() % 16 == 0 and v.is_cuda):
                v = v.to(table.device, torch.float32).contiguous()
                keep.append(v)
            srcs.append(v.data_ptr())
        ext.cache_write(srcs, [int(s) for s, _, _ in part], [int(c) for _, _, c in part], table, ctx)
    # (converted copies in ``keep`` may be freed now: the caching allocator hands their blocks only
    # to work queued after these launches on the same stream)


def masked_cosine_argmax(q: torch.Tensor, table: torch.Tensor, norms: torch.Tensor, ctx: torch.Tensor, cid: int,
                         thr: float) -> Tuple[int, float]:
    """Best row of ``table`` with ctx id == cid and cosine >= thr -> (row, sim) or (-1, 0.0) (one
    query: ``cache_scan``; on the GPU the row norms are computed in the kernel, ``norms`` is the
    host table's and is only used by the CPU reference)."""
    ext = _native(table)
    if ext is None:
        return ref.masked_cosine_argmax(q, table, norms, ctx, cid, thr)
    return cache_scan([q.reshape(-1)], [cid], table, ctx, table.shape[0], thr)[0]


from .gemm import autotune as gemm_autotune, linear, linear_swiglu, norm_linear  # noqa: E402


def step_fetch(dec_host: torch.Tensor, dec_dev: torch.Tensor, ids_off: int, src_off: int, n_ids: int,
               d_out: torch.Tensor, items_host: Optional[torch.Tensor] = None,
               items_dev: Optional[torch.Tensor] = None) -> None:
    """Decode-step inputs from a pinned host buffer into ``dec_dev`` by a kernel (graph-capturable,
    no copy engine): ``dec_dev[:] = dec_host`` except ids ``[ids_off, ids_off + n_ids)``, which take
    ``d_out[src[i]]`` where ``src[i] = dec_host[src_off + i] >= 0`` (the previous step's tokens);
    and the work list ``items_dev <- items_host`` (its header's length)."""
    ext = _native(dec_dev)
    if ext is None:
        h = dec_host.to(dec_dev.device)
        src = h[src_off:src_off + n_ids].long()
        ids = h[ids_off:ids_off + n_ids].clone()
        m = (src >= 0) & (src < n_ids)
        ids[m] = d_out[src[m]].to(ids.dtype)
        dec_dev.copy_(h)
        dec_dev[ids_off:ids_off + n_ids] = ids
        if items_host is not None:
            n = work_items_len(items_host.numpy())
            items_dev[:n].copy_(items_host[:n])
        return
    ext.step_fetch(dec_host, dec_dev, int(ids_off), int(src_off), int(n_ids), d_out, items_host, items_dev)


def step_store(d_out: torch.Tensor, out_host: torch.Tensor, n: int) -> None:
    """``out_host[:n] = d_out[:n]`` by a kernel writing the pinned host buffer (graph-capturable)."""
    ext = _native(d_out)
    if ext is None:
        out_host[:n].copy_(d_out[:n])
        return
    ext.step_store(d_out, out_host, int(n))


def scatter_pairs(dst: torch.Tensor, buf: torch.Tensor) -> None:
    """dst.view(-1)[idx_i] = val_i for buf = [n, idx0, val0, idx1, val1, ...] (int32)."""
    ext = _native(dst)
    if ext is None:
        n = int(buf[0])
        if n:
            pairs = buf[1:1 + 2 * n].view(-1, 2).long()
            dst.view(-1)[pairs[:, 0]] = pairs[:, 1].to(dst.dtype)
        return
    ext.scatter_pairs(dst, buf)
