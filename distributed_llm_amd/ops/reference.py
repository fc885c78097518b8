"""Plain-PyTorch (f32 math) reference implementations of every kernel in csrc/kernels.

Used (a) on CPU tensors (tests, CPU-only runs) and (b) as the numerics oracle the GPU kernel
tests compare against.  Layout contracts are identical to the HIP kernels.
"""
from __future__ import annotations

import math
from typing import List, Optional, Tuple

import torch

BS = 16


def rms_norm(x, w, eps, residual=None):
    if residual is not None:
        r = (x.float() + residual.float()).to(x.dtype)
        residual.copy_(r)
        x = r
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()
    return y.to(x.dtype)


def layer_norm(x, w, b, eps, residual=None):
    if residual is not None:
        r = (x.float() + residual.float()).to(x.dtype)
        residual.copy_(r)
        x = r
    y = torch.nn.functional.layer_norm(x.float(), (x.shape[-1],), w.float(), b.float(), eps)
    return y.to(x.dtype)


def llama3_scale_inv_freq(inv: torch.Tensor, sc: dict) -> torch.Tensor:
    factor = sc.get("factor", 8.0)
    lo = sc.get("low_freq_factor", 1.0)
    hi = sc.get("high_freq_factor", 4.0)
    old = sc.get("original_max_position_embeddings", 8192)
    wl = 2 * math.pi / inv
    lo_wl, hi_wl = old / lo, old / hi
    out = torch.where(wl > lo_wl, inv / factor, inv)
    smooth = (old / wl - lo) / (hi - lo)
    mid = (1 - smooth) * inv / factor + smooth * inv
    is_mid = (wl <= lo_wl) & (wl >= hi_wl)
    return torch.where(is_mid, mid, out)


def _rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    # x [T, h, d] f32; cos/sin [T, d/2]
    h = x.shape[-1] // 2
    x1, x2 = x[..., :h], x[..., h:]
    c, s = cos[:, None, :], sin[:, None, :]
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1)


def rope_and_cache(qkv, positions, cos_sin, slots, k_cache, v_cache, nq, nkv, d):
    T = qkv.shape[0]
    f = qkv[:, : (nq + 2 * nkv) * d].float()
    q = f[:, : nq * d].view(T, nq, d)
    k = f[:, nq * d:(nq + nkv) * d].view(T, nkv, d)
    v = qkv[:, (nq + nkv) * d:(nq + 2 * nkv) * d].view(T, nkv, d)
    cs = cos_sin[positions.long()].float()
    cos, sin = cs[:, : d // 2], cs[:, d // 2:]
    q = _rope(q, cos, sin).to(qkv.dtype)
    k = _rope(k, cos, sin).to(qkv.dtype)
    kv_write(k, v, slots, k_cache, v_cache)
    return q.contiguous()


def kv_write(k, v, slots, k_cache, v_cache):
    sl = slots.long()
    ok = sl >= 0
    if not bool(ok.any()):
        return
    sl, k, v = sl[ok], k[ok], v[ok]
    blk, off = sl // BS, sl % BS
    k_cache[blk, :, off, :] = k.to(k_cache.dtype)
    v_cache[blk, :, :, off] = v.to(v_cache.dtype)


def write_newest_v(v_new, v_cache, block_tables, seq_qstart, seq_ctx):
    """Decode hand-over (attention.hip AttnArgs.v_new): each sequence's newest key ctx - 1 takes V
    row ``v_new[qstart]`` ([T, nkv * d] row-major) in the V^T cache."""
    nkv, d = v_cache.shape[1], v_cache.shape[2]
    for s in range(block_tables.shape[0]):
        ctx, qs = int(seq_ctx[s]), int(seq_qstart[s])
        if ctx <= 0:
            continue
        key = ctx - 1
        blk = int(block_tables[s, key // BS])
        v_cache[blk, :, :, key % BS] = v_new[qs].view(nkv, d).to(v_cache.dtype)


def gather_kv(k_cache, v_cache, block_table, n):
    """Dense K, V [n, nkv, d] of one sequence from the paged caches."""
    nb = (n + BS - 1) // BS
    blocks = block_table[:nb].long()
    k = k_cache[blocks]                       # [nb, nkv, 16, d]
    v = v_cache[blocks].transpose(2, 3)       # [nb, nkv, 16, d]
    k = k.permute(0, 2, 1, 3).reshape(nb * BS, k.shape[1], k.shape[3])[:n]
    v = v.permute(0, 2, 1, 3).reshape(nb * BS, v.shape[1], v.shape[3])[:n]
    return k, v


def paged_attention(q, k_cache, v_cache, block_tables, seq_qstart, seq_qlen, seq_ctx, scale, causal=True):
    out = torch.zeros_like(q)
    nq, d = q.shape[1], q.shape[2]
    nkv = k_cache.shape[1]
    G = nq // nkv
    for s in range(block_tables.shape[0]):
        ql, ctx, qs = int(seq_qlen[s]), int(seq_ctx[s]), int(seq_qstart[s])
        if ql == 0 or ctx == 0:
            continue
        k, v = gather_kv(k_cache, v_cache, block_tables[s], ctx)
        k = k.float().repeat_interleave(G, dim=1)  # [ctx, nq, d]
        v = v.float().repeat_interleave(G, dim=1)
        qq = q[qs:qs + ql].float()                 # [ql, nq, d]
        sc = torch.einsum("qhd,khd->hqk", qq, k) * scale
        if causal:
            pos = torch.arange(ctx - ql, ctx, device=q.device)[:, None]
            keys = torch.arange(ctx, device=q.device)[None, :]
            sc = sc.masked_fill((keys > pos)[None], float("-inf"))
        p = torch.softmax(sc, dim=-1)
        o = torch.einsum("hqk,khd->qhd", p, v)
        out[qs:qs + ql] = o.to(q.dtype)
    return out


def silu_mul(gu):
    I = gu.shape[1] // 2
    g, u = gu[:, :I].float(), gu[:, I:].float()
    return (torch.nn.functional.silu(g) * u).to(gu.dtype)


def gelu(x):
    return torch.nn.functional.gelu(x.float()).to(x.dtype)


def encoder_attention(qkv, lens, B, S, nh, d, scale):
    """Bidirectional attention of a padded batch: qkv [B*S, 3 nh d] -> [B*S, nh d]; keys >= lens[b]
    masked (csrc/kernels/encoder.hip)."""
    x = qkv.float().view(B, S, 3, nh, d).permute(2, 0, 3, 1, 4)   # [3, B, nh, S, d]
    q, k, v = x[0], x[1], x[2]
    s = (q @ k.transpose(-1, -2)) * scale
    keymask = torch.arange(S, device=qkv.device)[None, :] < lens.to(qkv.device).long()[:, None]
    s = s.masked_fill(~keymask[:, None, None, :], float("-inf"))
    p = torch.softmax(s, dim=-1).nan_to_num(0.0)
    o = (p @ v).permute(0, 2, 1, 3).reshape(B * S, nh * d)
    return o.to(qkv.dtype)


def embed_ln(ids, word, pos, type0, w, b, S, eps):
    """LayerNorm(word[ids] + pos[t % S] + type0) for flattened [B*S] ids (csrc/kernels/encoder.hip)."""
    T = ids.numel()
    p = pos[:S].float().repeat(T // S, 1)
    x = word[ids.long().reshape(-1)].float() + p + type0.float()
    y = torch.nn.functional.layer_norm(x, (x.shape[-1],), w.float(), b.float(), eps)
    return y.to(word.dtype)


def mean_pool_l2(x, lens):
    B, S, H = x.shape
    m = (torch.arange(S)[None, :].to(x.device) < lens.to(x.device)[:, None]).float()
    s = (x.float() * m[..., None]).sum(1) / m.sum(1, keepdim=True).clamp(min=1.0)
    return torch.nn.functional.normalize(s, dim=-1, eps=1e-12)


def moe_gate(logits, k):
    lf = logits.float()
    vals, ids = torch.topk(lf, k, dim=-1)
    w = torch.softmax(vals, dim=-1)
    return ids.to(torch.int32), w


def moe_ffn(x, ids, wts, w13, w2):
    """sum_j wts[t, j] * (silu(x w13_e[:I]^T) * (x w13_e[I:]^T)) w2_e^T  with e = ids[t, j] (f32 math,
    bf16 rounding of the activation like the kernel)."""
    T, H = x.shape
    I = w13.shape[1] // 2
    out = torch.zeros((T, H), dtype=torch.float32, device=x.device)
    xf = x.float()
    for j in range(ids.shape[1]):
        for e in ids[:, j].unique().tolist():
            sel = (ids[:, j] == e).nonzero().flatten()
            gu = xf[sel] @ w13[e].float().t()
            act = (torch.nn.functional.silu(gu[:, :I]) * gu[:, I:]).to(x.dtype).float()
            out[sel] += wts[sel, j:j + 1].float() * (act @ w2[e].float().t())
    return out.to(x.dtype)


def sample_top_p(vals, idx, temperature, top_p, uniform):
    t = temperature.float().clamp(min=1e-5)[:, None]
    p = torch.softmax(vals.float() / t, dim=-1)
    c = torch.cumsum(p, dim=-1)
    # keep the smallest prefix whose mass reaches top_p
    keep = (c - p) < top_p.float()[:, None]
    keep[:, 0] = True
    p = p * keep
    p = p / p.sum(-1, keepdim=True)
    cdf = torch.cumsum(p, dim=-1)
    pick = torch.searchsorted(cdf, uniform.float()[:, None].clamp(max=0.999999), right=True).clamp(max=vals.shape[1] - 1)
    return torch.gather(idx, 1, pick).view(-1).to(torch.int32)


def row_uniform(seed: int, rows: int) -> torch.Tensor:
    """Counter-based uniforms u[row] in [0, 1) — the same hash as sample_rows_kernel."""
    M = 0xFFFFFFFF
    out = []
    for r in range(rows):
        h = (seed + r * 0x9E3779B9) & M
        h ^= h >> 16
        h = (h * 0x7FEB352D) & M
        h ^= h >> 15
        h = (h * 0x846CA68B) & M
        h ^= h >> 16
        out.append((h >> 8) / 16777216.0)
    return torch.tensor(out, dtype=torch.float32)


def sample_rows(logits, temperature, top_p, top_k, seed: int):
    """Reference of the fused row sampler: greedy rows -> arg-max (lowest index on ties); sampled
    rows -> top-k (value desc, index asc; k <= 0 -> 256) -> temperature -> nucleus -> draw."""
    lg = logits.float()
    B, V = lg.shape
    u = row_uniform(int(seed) & 0xFFFFFFFF, B)
    out = torch.empty(B, dtype=torch.int32)
    for r in range(B):
        t = float(temperature[r])
        if not t > 0.0:
            out[r] = int(torch.argmax(lg[r]))
            continue
        k = int(top_k[r])
        k = 256 if k <= 0 or k > 256 else k
        k = min(k, V)
        order = sorted(range(V), key=lambda i: (-float(lg[r, i]), i))[:k]
        vals = lg[r, order]
        w = torch.exp((vals - vals[0]) / max(t, 1e-5))
        c = torch.cumsum(w, 0)
        s = float(c[-1])
        cut = k
        for i in range(k):
            if float(c[i]) >= float(top_p[r]) * s:
                cut = i + 1
                break
        target = float(u[r]) * float(c[cut - 1])
        pick = cut - 1
        for i in range(cut):
            if float(c[i]) > target:
                pick = i
                break
        out[r] = order[pick]
    return out


def _draw_ranked(vals, ids, t: float, top_p: float, k: int, u: float) -> int:
    """sample_rows' draw over candidates already ranked (value desc, id asc)."""
    if not t > 0.0:
        return int(ids[0])
    k = 256 if k <= 0 or k > 256 else k
    k = min(k, len(ids))
    vals = torch.as_tensor(vals[:k], dtype=torch.float32)
    w = torch.exp((vals - vals[0]) / max(t, 1e-5))
    c = torch.cumsum(w, 0)
    s = float(c[-1])
    cut = k
    for i in range(k):
        if float(c[i]) >= top_p * s:
            cut = i + 1
            break
    target = u * float(c[cut - 1])
    pick = cut - 1
    for i in range(cut):
        if float(c[i]) > target:
            pick = i
            break
    return int(ids[pick])


def tp_candidates(logits, start: int, kc: int = 256):
    """Reference of tp_cands_kernel: [S, kc, 2] int32 (value f32 bits, global id)."""
    lg = logits.float().cpu()
    S, V = lg.shape
    out = torch.empty((S, kc, 2), dtype=torch.int32)
    out[:, :, 0] = torch.tensor([float("-inf")], dtype=torch.float32).view(torch.int32)
    out[:, :, 1] = 2 ** 31 - 1
    _, order = torch.sort(-lg, dim=1, stable=True)          # value desc, index asc
    n = min(kc, V)
    for r in range(S):
        idx = order[r, :n]
        out[r, :n, 0] = lg[r, idx].contiguous().view(torch.int32)
        out[r, :n, 1] = (idx + start).to(torch.int32)
    return out.to(logits.device)


def tp_sample(cands, temperature, top_p, top_k, seed: int):
    """Reference of tp_sample_kernel over all-gathered candidates [tp, S, kc, 2]."""
    c = cands.cpu()
    tp, S, kc, _ = c.shape
    u = row_uniform(int(seed) & 0xFFFFFFFF, S)
    out = torch.empty(S, dtype=torch.int32)
    for r in range(S):
        v = c[:, r, :, 0].reshape(-1).contiguous().view(torch.float32)
        ids = c[:, r, :, 1].reshape(-1)
        keep = ids != 2 ** 31 - 1
        v, ids = v[keep], ids[keep]
        order = sorted(range(len(ids)), key=lambda i: (-float(v[i]), int(ids[i])))
        out[r] = _draw_ranked([float(v[i]) for i in order], [int(ids[i]) for i in order], float(temperature[r]),
                              float(top_p[r]), int(top_k[r]), float(u[r]))
    return out


def cosine_scores(q, c):
    qn = q.float()
    cn = c.float()
    num = qn @ cn.T
    den = qn.norm(dim=-1, keepdim=True) * cn.norm(dim=-1)[None, :]
    return torch.where(den < 1e-9, torch.zeros_like(num), num / den.clamp(min=1e-30))


def masked_cosine_argmax(q, table, norms, ctx, cid, thr) -> Tuple[int, float]:
    qf = q.float().reshape(-1)
    nq = float(qf.norm())
    if nq < 1e-9 or table.shape[0] == 0:
        return -1, 0.0
    mask = (ctx == cid) & (norms >= 1e-9)
    if not bool(mask.any()):
        return -1, 0.0
    sims = (table.float() @ qf) / (norms.float().clamp(min=1e-30) * nq)
    sims = torch.where(mask, sims, torch.full_like(sims, -float("inf")))
    j = int(torch.argmax(sims))
    s = float(sims[j])
    return (j, s) if s >= thr else (-1, 0.0)


def cache_scan(queries, cids, table, ctx, n_rows, thr) -> List[Tuple[int, float]]:
    """fp32 reference of ops.cache_scan: per query, the row of its context id with the highest
    cosine >= thr (lowest row on ties; rows or queries of norm < 1e-9 never match) or (-1, 0.0)."""
    t = table[:n_rows].float()
    c = ctx[:n_rows]
    rn = t.norm(dim=-1)
    out = []
    for q, cid in zip(queries, cids):
        qf = q.float().reshape(-1)
        nq = float(qf.norm())
        mask = (c == int(cid)) & (rn >= 1e-9)
        if nq < 1e-9 or not bool(mask.any()):
            out.append((-1, 0.0))
            continue
        sims = (t @ qf) / (rn.clamp(min=1e-30) * nq)
        sims = torch.where(mask, sims, torch.full_like(sims, -float("inf")))
        j = int(torch.argmax(sims))
        s = float(sims[j])
        out.append((j, s) if s >= thr else (-1, 0.0))
    return out


def embedding(ids, table, lo=0):
    """fp32-free reference of ops.embedding (exact row copies, zero rows outside the shard)."""
    local = ids.reshape(-1).long() - lo
    ok = (local >= 0) & (local < table.shape[0])
    return table[local.clamp(0, table.shape[0] - 1)] * ok.unsqueeze(-1).to(table.dtype)
