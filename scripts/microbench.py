"""Engine/kernel micro-benchmarks on one GPU (prints JSON lines).

  decode  : one hipGraph decode step of the flagship model at batch B, context C
            (weight bytes + KV bytes per step -> effective HBM bandwidth)
  attn    : paged decode attention kernel alone (KV bytes / time)
  prefill : packed prefill throughput (tokens/s) for a batch of prompts
"""
import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from distributed_llm_amd import ops
from distributed_llm_amd.engine.llm_engine import LLMEngine


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def bench_attn_dyn(B, C, nq, nkv, d, z, target, var=True):
    """Dynamic split-K (engine decode path): split length from the batch's total context."""
    g = torch.Generator().manual_seed(0)
    ctxs = (torch.randint(C // 4, 7 * C // 4 + 1, (B,), generator=g).tolist() if var else [C] * B)
    Cm = max(ctxs)
    NB = B * ((Cm + 15) // 16) + 8
    kc = torch.randn(NB, nkv, 16, d, device="cuda").to(torch.bfloat16)
    vc = torch.randn(NB, nkv, d, 16, device="cuda").to(torch.bfloat16)
    nb = (Cm + 15) // 16
    bt = torch.randperm(NB - 8, device="cuda")[:B * nb].view(B, nb).to(torch.int32)
    q = torch.randn(B, nq, d, device="cuda").to(torch.bfloat16)
    I = lambda x: torch.tensor(x, dtype=torch.int32, device="cuda")
    qs, ql, cx = I(list(range(B))), I([1] * B), I(ctxs)
    ts, tt = ops.build_tiles([1] * B, nq // nkv)
    ts, tt = I(ts), I(tt)
    sl = int(max(256, math.ceil(sum(ctxs) * nkv / target / 256) * 256))
    slt = I([sl])
    ms = timeit(lambda: ops.paged_attention(q, kc, vc, bt, qs, ql, cx, ts, tt, splits=z, split_len=slt))
    # correctness against the single-split kernel
    ref_o = ops.paged_attention(q, kc, vc, bt, qs, ql, cx, ts, tt, splits=1)
    got = ops.paged_attention(q, kc, vc, bt, qs, ql, cx, ts, tt, splits=z, split_len=slt)
    err = (ref_o.float() - got.float()).abs().max().item()
    kv_bytes = sum(ctxs) * nkv * d * 2 * 2
    return {"bench": "attn_decode_dyn", "B": B, "C": sum(ctxs) // B, "var": var, "nq": nq, "nkv": nkv, "d": d,
            "z": z, "target": target, "split_len": sl, "us": round(ms * 1000, 1),
            "GBps": round(kv_bytes / ms / 1e6, 1), "max_err_vs_1split": err}


def bench_attn_wl(B, C, nq, nkv, d, grid, per_wg, var=True, min_chunk=256, waves="auto"):
    """Persistent work-list decode attention (engine default): tiles longest context first."""
    import numpy as np
    g = torch.Generator().manual_seed(0)
    ctxs = (torch.randint(C // 4, 7 * C // 4 + 1, (B,), generator=g).tolist() if var else [C] * B)
    Cm = max(ctxs)
    NB = B * ((Cm + 15) // 16) + 8
    kc = torch.randn(NB, nkv, 16, d, device="cuda").to(torch.bfloat16)
    vc = torch.randn(NB, nkv, d, 16, device="cuda").to(torch.bfloat16)
    nb = (Cm + 15) // 16
    bt = torch.randperm(NB - 8, device="cuda")[:B * nb].view(B, nb).to(torch.int32)
    q = torch.randn(B, nq, d, device="cuda").to(torch.bfloat16)
    I = lambda x: torch.tensor(x, dtype=torch.int32, device="cuda")
    qs, ql, cx = I(list(range(B))), I([1] * B), I(ctxs)
    order = np.argsort(-np.array(ctxs), kind="stable")
    ts, tt = I(order.astype(np.int32).tolist()), I([0] * B)
    z = 16
    ws = (torch.empty(B * nkv * z * 16 * d, device="cuda"), torch.empty(B * nkv * z * 16 * 2, device="cuda"),
          torch.zeros(B * nkv + 2, dtype=torch.int32, device="cuda"))
    items = ops.decode_work_items(np.array(ctxs)[order], nkv, z, per_wg * grid, min_chunk=min_chunk)
    it = torch.tensor(items, device="cuda")
    run = lambda: ops.paged_attention(q, kc, vc, bt, qs, ql, cx, ts, tt, splits=z, workspace=ws, items=it,
                                      grid_items=grid)
    ms = timeit(run)
    ref_o = ops.paged_attention(q, kc, vc, bt, qs, ql, cx, ts, tt, splits=1)
    err = (ref_o.float() - run().float()).abs().max().item()
    kv_bytes = sum(ctxs) * nkv * d * 2 * 2
    return {"bench": "attn_decode_worklist", "B": B, "C": sum(ctxs) // B, "var": var, "nq": nq, "nkv": nkv,
            "d": d, "grid": grid, "per_wg": per_wg, "items": int(items[0]), "min_chunk": min_chunk,
            "waves": os.environ.get("DLLM_ATTN_WAVES", "auto"), "us": round(ms * 1000, 1),
            "GBps": round(kv_bytes / ms / 1e6, 1), "max_err_vs_1split": err}


def bench_attn(B, C, nq, nkv, d, splits, var=False):
    """var=True: contexts uniform in [C/4, 7C/4] (mean C) like a serving batch, else all C."""
    g = torch.Generator().manual_seed(0)
    ctxs = (torch.randint(C // 4, 7 * C // 4 + 1, (B,), generator=g).tolist() if var else [C] * B)
    C = max(ctxs)
    NB = B * ((C + 15) // 16) + 8
    kc = torch.randn(NB, nkv, 16, d, device="cuda").to(torch.bfloat16)
    vc = torch.randn(NB, nkv, d, 16, device="cuda").to(torch.bfloat16)
    nb = (C + 15) // 16
    bt = torch.randperm(NB - 8, device="cuda")[:B * nb].view(B, nb).to(torch.int32)
    q = torch.randn(B, nq, d, device="cuda").to(torch.bfloat16)
    I = lambda x: torch.tensor(x, dtype=torch.int32, device="cuda")
    qs, ql, cx = I(list(range(B))), I([1] * B), I(ctxs)
    ts, tt = ops.build_tiles([1] * B, nq // nkv)
    ts, tt = I(ts), I(tt)
    ms = timeit(lambda: ops.paged_attention(q, kc, vc, bt, qs, ql, cx, ts, tt, splits=splits))
    kv_bytes = sum(ctxs) * nkv * d * 2 * 2
    return {"bench": "attn_decode", "B": B, "C": sum(ctxs) // B, "var": var, "nq": nq, "nkv": nkv, "d": d,
            "splits": splits, "waves": os.environ.get("DLLM_ATTN_WAVES", "auto"),
            "us": round(ms * 1000, 1), "GBps": round(kv_bytes / ms / 1e6, 1)}


def bench_decode(eng, B, C):
    # fabricate B running sequences of context C (tokens are irrelevant for timing)
    bm = eng.bm
    seqs = []
    for i in range(B):
        sid = 10_000_000 + i
        tbl, _ = bm.allocate(sid, [5 + (i % 1000)] + [5] * (C - 1))
        if not tbl:
            raise RuntimeError(f"KV cache too small for B={B} x C={C} (set MB_KV_GB)")
        row = eng._free_rows.pop()
        t = bm.block_table(sid)
        eng.bt_host[row, :len(t)] = t
        seqs.append((sid, row))
    eng._bt_dirty = True

    class S:  # minimal stand-in for engine._Seq
        pass
    run = []
    for sid, row in seqs:
        s = S()
        s.id, s.row, s.out = sid, row, [7]
        s.length = C
        run.append(s)
    bs = eng._bucket(B)
    o, h, R = eng._off, eng.dec_host, eng.R
    import numpy as np
    rows = np.array([s.row for s in run])
    pos = np.full(B, C - 1)
    blocks = eng.bt_host[rows, pos // 16]
    h[:] = 0
    if len(o) > 9:
        h[o[9]:o[9] + bs] = -1     # input ids from this buffer, not gathered from d_out
    h[o[0]:o[0] + B] = 7
    h[o[1]:o[1] + B] = pos
    h[o[2]:o[2] + bs] = -1
    h[o[2]:o[2] + B] = blocks * 16 + pos % 16
    h[o[3]:o[3] + bs] = R
    h[o[3]:o[3] + B] = rows
    h[o[4] + rows] = np.arange(B)
    h[o[5] + rows] = 1
    h[o[6] + rows] = C
    t = float(os.environ.get("MB_TEMP", "0"))   # > 0: sampled rows (top-k 40, top-p 0.9), else greedy
    if t > 0:
        s0, mb, hf = eng._so, eng.buckets[-1], eng.dec_host_f
        hf[s0:s0 + bs] = t
        hf[s0 + mb:s0 + mb + bs] = 0.9
        h[s0 + 2 * mb:s0 + 2 * mb + bs] = 40
    eng._sync_bt()
    eng.dec_dev.copy_(eng.dec_host_t)
    if eng._use_worklist(bs):
        # the persistent attention kernel walks a host-built work list: without it the step's
        # attention launches would find zero units (rounds before r2-late measured that by mistake)
        items_t, items = eng._items_bufs[0]
        ops.decode_work_items(np.full(B, C), eng.model.nkv, eng.max_splits,
                              eng.ATTN_ITEMS_PER_WG * eng._attn_grid(bs), min_chunk=eng.ATTN_MIN_CHUNK, out=items,
                              seq=rows, qstart=np.arange(B))
        n_items = ops.work_items_len(items)
        eng.items_dev[:n_items].copy_(items_t[:n_items])
    g = eng._graphs.get(eng._gkey(bs, 0)) or eng._capture(bs, 0)
    ms = timeit(g.replay)
    wbytes = eng.model.weight_bytes()
    kv = B * C * eng.cfg.n_layers * eng.model.nkv * eng.model.d * 2 * 2
    for sid, row in seqs:
        bm.free(sid)
        eng.bt_host[row] = 0
        eng._free_rows.append(row)
    return {"bench": "decode_step", "model": eng.cfg.name, "B": B, "bucket": bs, "C": C, "ms": round(ms, 3),
            "tok_s": round(B / ms * 1000, 1), "weight_GB": round(wbytes / 1e9, 2),
            "eff_GBps": round((wbytes + kv) / ms / 1e6, 1)}


def bench_prefill(eng, B, L):
    from distributed_llm_amd.engine.sampling import SamplingParams
    import random
    prompts = [[random.randint(3, 250) for _ in range(L)] for _ in range(B)]
    eng.bm.reset()
    t = time.perf_counter()
    eng.generate(prompts, SamplingParams(max_new_tokens=1))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    return {"bench": "prefill", "B": B, "L": L, "s": round(dt, 4), "tok_s": round(B * L / dt, 1)}


def bench_moe(T, H=4096, I=14336, E=8, k=2, plan=None):
    """Mixtral expert FFN: the old per-wave kernel (moe_ffn) vs the grouped tgemm (moe_ffn_tg).
    Bytes = the weights of the experts the batch touches (+ activations); FLOPs = 6 T k H I."""
    from distributed_llm_amd.models.llama import gate_up_order
    g = torch.Generator(device="cuda").manual_seed(T)
    w13 = (torch.randn(E, 2 * I, H, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
    w2 = (torch.randn(E, H, I, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
    w13i = w13.index_select(1, gate_up_order(I).cuda()).contiguous()
    x = (torch.randn(T, H, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
    ids, w = ops.moe_gate(torch.randn(T, E, device="cuda", generator=g), k)
    touched = len(set(ids.flatten().tolist()))
    wbytes = touched * 3 * H * I * 2
    flops = 6.0 * T * k * H * I
    res = {"bench": "moe_ffn", "T": T, "H": H, "I": I, "E": E, "k": k, "experts_touched": touched}
    iters = 10 if T <= 512 else 3
    ms_old = timeit(lambda: ops.moe_ffn(x, ids, w, w13, w2), iters=iters, warm=2)
    ms_new = timeit(lambda: ops.moe_ffn_tg(x, ids, w, w13i, w2, plan), iters=iters, warm=2)
    for name, ms in (("old", ms_old), ("tg", ms_new)):
        res[f"{name}_us"] = round(ms * 1000, 1)
        res[f"{name}_weight_TBps"] = round(wbytes / ms / 1e9, 2)
        res[f"{name}_TFLOPs"] = round(flops / ms / 1e9, 1)
    err = (ops.moe_ffn_tg(x, ids, w, w13i, w2, plan).float() - ops.moe_ffn(x, ids, w, w13, w2).float()).abs().max()
    res["max_abs_diff_tg_vs_old"] = round(float(err), 5)
    res["plan"] = list(plan) if plan else "auto"
    del w13, w2, w13i
    torch.cuda.empty_cache()
    return res


def bench_post(M, N=11264, H=2048):
    """Standalone fused-op epilogues on a GEMM output y [M, N] (vendor-core split form)."""
    from distributed_llm_amd.ops import gemm as G
    ext = ops._native(torch.empty(1, device="cuda"))
    y = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    slots = G.max_slots(H)
    ssq = torch.rand(slots, M, device="cuda") + 1.0
    act = torch.empty(M, N // 2, device="cuda", dtype=torch.bfloat16)
    r = torch.randn(M, H, device="cuda").to(torch.bfloat16)
    h = torch.randn(M, H, device="cuda").to(torch.bfloat16)
    res = {"bench": "post", "M": M, "N": N, "H": H}
    for n_slots in (1, 32):
        us = G._time(lambda i: ext.swiglu_post(y, ssq, n_slots, 1.0 / H, 1e-5, act)) 
        res[f"swiglu_post_slots{n_slots}_us"] = round(us, 2)
    res["swiglu_post_GBps"] = round(M * N * 3 / res["swiglu_post_slots1_us"] / 1e3, 1)
    us = G._time(lambda i: ext.res_add_ssq(h, r, ssq))
    res["res_add_ssq_us"] = round(us, 2)
    return res


def bench_flash(L, nq, nkv, d, B=1):
    """Cold causal prefill of B prompts of L tokens: flash_prefill.hip vs the 16-row paged kernel.
    FLOPs = 4 * nq * d * (causal pairs) per prompt (QK^T and PV)."""
    import numpy as np
    g = torch.Generator(device="cuda").manual_seed(L + d)
    nb = (L + 15) // 16
    kc = (torch.randn(B * nb + 4, nkv, 16, d, device="cuda", generator=g)).to(torch.bfloat16)
    vc = (torch.randn(B * nb + 4, nkv, d, 16, device="cuda", generator=g)).to(torch.bfloat16)
    bt = (torch.randperm(B * nb, device="cuda", generator=g) + 1).view(B, nb).to(torch.int32)
    q = torch.randn(B * L, nq, d, device="cuda", generator=g).to(torch.bfloat16)
    I = lambda x: torch.tensor(x, dtype=torch.int32, device="cuda")
    qs, ql, cx = I([i * L for i in range(B)]), I([L] * B), I([L] * B)
    G = nq // nkv
    fts, ftt = ops.flash_tiles([L] * B, G)
    pts, ptt = ops.build_tiles([L] * B, G)
    fts, ftt, pts, ptt = I(fts), I(ftt), I(pts), I(ptt)
    it = 10 if L <= 4096 else 3
    ms_f = timeit(lambda: ops.flash_attention(q, kc, vc, bt, qs, ql, cx, fts, ftt), iters=it, warm=2)
    ms_p = timeit(lambda: ops.paged_attention(q, kc, vc, bt, qs, ql, cx, pts, ptt, xcd_remap=True), iters=it, warm=2)
    a = ops.flash_attention(q, kc, vc, bt, qs, ql, cx, fts, ftt)
    b = ops.paged_attention(q, kc, vc, bt, qs, ql, cx, pts, ptt, xcd_remap=True)
    flops = 4.0 * nq * d * (L * (L + 1) / 2) * B
    return {"bench": "flash_prefill", "B": B, "L": L, "nq": nq, "nkv": nkv, "d": d,
            "flash_us": round(ms_f * 1000, 1), "flash_TFLOPs": round(flops / ms_f / 1e9, 1),
            "paged16_us": round(ms_p * 1000, 1), "paged16_TFLOPs": round(flops / ms_p / 1e9, 1),
            "speedup": round(ms_p / ms_f, 2), "max_abs_diff": round(float((a.float() - b.float()).abs().max()), 4)}


def bench_flash_cached(Q, C, nq, nkv, d):
    """One prompt's new tokens behind a cached history (a conversation turn with a prefix hit):
    Q query tokens at the end of a C-key context, causal; split-KV auto (max_ctx given) vs off."""
    g = torch.Generator(device="cuda").manual_seed(Q + C + d)
    nb = (C + 15) // 16
    kc = (torch.randn(nb + 4, nkv, 16, d, device="cuda", generator=g)).to(torch.bfloat16)
    vc = (torch.randn(nb + 4, nkv, d, 16, device="cuda", generator=g)).to(torch.bfloat16)
    bt = (torch.randperm(nb, device="cuda", generator=g) + 1).view(1, nb).to(torch.int32)
    q = torch.randn(Q, nq, d, device="cuda", generator=g).to(torch.bfloat16)
    I = lambda x: torch.tensor(x, dtype=torch.int32, device="cuda")
    qs, ql, cx = I([0]), I([Q]), I([C])
    fts, ftt = ops.flash_tiles([Q], nq // nkv)
    fts, ftt = I(fts), I(ftt)
    run = lambda mc: ops.flash_attention(q, kc, vc, bt, qs, ql, cx, fts, ftt, max_ctx=mc)
    ms_s = timeit(lambda: run(C), iters=10, warm=2)
    ms_1 = timeit(lambda: run(0), iters=10, warm=2)
    diff = float((run(C).float() - run(0).float()).abs().max())
    flops = 4.0 * nq * d * Q * C
    return {"bench": "flash_cached", "Q": Q, "C": C, "nq": nq, "nkv": nkv, "d": d,
            "splits": ops.flash_splits(len(fts) * nkv, C), "split_us": round(ms_s * 1000, 1),
            "nosplit_us": round(ms_1 * 1000, 1), "split_TFLOPs": round(flops / ms_s / 1e9, 1),
            "nosplit_TFLOPs": round(flops / ms_1 / 1e9, 1), "max_abs_diff": round(diff, 4)}


def bench_gemm(M, N, K):
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    ms = timeit(lambda: torch.nn.functional.linear(x, w), iters=50)
    return {"bench": "gemm_hipblaslt", "M": M, "N": N, "K": K, "us": round(ms * 1000, 1),
            "weight_GBps": round(N * K * 2 / ms / 1e6, 1), "TFLOPs": round(2 * M * N * K / ms / 1e9, 1)}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="tinyllama-1.1b")
    ap.add_argument("--what", default="gemm,attn,decode,prefill")
    a = ap.parse_args()
    what = a.what.split(",")
    if "tune" in what:
        from distributed_llm_amd.ops import gemm as G
        shapes = [(2560, 2048, False), (2048, 2048, False), (11264, 2048, False), (2048, 5632, True),
                  (32000, 2048, False), (6144, 4096, False), (4096, 4096, False), (28672, 4096, False), (4096, 14336, True)]
        ms = [int(x) for x in os.environ.get("MB_TUNE_M", "1,8,32,64,128,256,384,512").split(",")]
        if os.environ.get("MB_TUNE_SHAPES"):
            shapes = [tuple(int(v) for v in t.split("x")) + (False,) for t in os.environ["MB_TUNE_SHAPES"].split(",")]
        G.autotune(shapes, ms, "cuda", verbose=True)
    if "flash_cached" in what:
        for (nq, nkv, d) in ((32, 4, 64), (32, 8, 128)):
            for (Q, C) in ((130, 2048), (130, 4096), (130, 16384), (512, 16384), (1024, 32768)):
                print(json.dumps(bench_flash_cached(Q, C, nq, nkv, d)), flush=True)
    if "flash" in what:
        for (nq, nkv, d) in ((32, 4, 64), (32, 8, 128), (32, 32, 96)):
            for L in (1024, 4096, 16384):
                print(json.dumps(bench_flash(L, nq, nkv, d)), flush=True)
            print(json.dumps(bench_flash(2048, nq, nkv, d, B=8)), flush=True)
    if "post" in what:
        for M in (64, 512, 2048, 4096):
            print(json.dumps(bench_post(M)), flush=True)
    if "moe" in what:
        Ts = [int(x) for x in os.environ.get("MB_MOE_T", "1,16,64,256,1024,4096").split(",")]
        for T in Ts:
            print(json.dumps(bench_moe(T)), flush=True)
        plans = {16: ((64, 128, 3, 1, 4, 64, 6, 1, 4), (64, 128, 6, 1, 4, 64, 6, 1, 4), (64, 128, 4, 1, 4, 128, 4, 1, 4),
                      (64, 64, 6, 1, 4, 64, 6, 1, 4)),
                 64: ((64, 128, 3, 1, 4, 64, 6, 1, 4), (64, 128, 6, 1, 4, 64, 6, 1, 4), (64, 128, 4, 1, 4, 128, 4, 1, 4)),
                 256: ((128, 128, 3, 1, 8, 128, 3, 1, 8), (128, 128, 4, 1, 8, 128, 4, 1, 8)),
                 4096: ((256, 256, 2, 1, 8, 128, 3, 1, 8), (128, 128, 4, 1, 8, 128, 4, 1, 8))}
        for T in [int(x) for x in os.environ.get("MB_MOE_PLAN_T", "16,64,256,4096").split(",")]:
            for plan in plans[T]:
                print(json.dumps(bench_moe(T, plan=plan)), flush=True)
    if "gemm" in what:
        for M in (1, 16, 64, 128, 256):
            for (N, K) in [(2560, 2048), (2048, 2048), (11264, 2048), (2048, 5632), (32000, 2048), (6144, 4096), (28672, 4096), (4096, 14336)]:
                print(json.dumps(bench_gemm(M, N, K)), flush=True)
    if "attn" in what:
        for (B, C, var) in [(1, 2048, False), (16, 2048, False), (64, 512, False), (64, 2048, False),
                            (64, 8192, False), (256, 1024, False), (256, 2048, True), (128, 2048, True)]:
            for (nq, nkv, d) in [(32, 4, 64), (32, 8, 128)]:
                for splits in (1, 2, 4, 8):
                    print(json.dumps(bench_attn(B, C, nq, nkv, d, splits, var)), flush=True)
    if "attn_dyn" in what:
        for (B, C, var) in [(1, 2048, False), (16, 2048, False), (64, 2048, True), (128, 2021, True),
                            (256, 1024, False), (256, 2034, True), (256, 4000, True)]:
            for (nq, nkv, d) in [(32, 4, 64), (32, 8, 128)]:
                print(json.dumps(bench_attn(B, C, nq, nkv, d, 1, var)), flush=True)
                for z in (4, 8):
                    for target in (1024, 2048, 4096):
                        print(json.dumps(bench_attn_dyn(B, C, nq, nkv, d, z, target, var)), flush=True)
    if "attn_wl" in what:
        for (B, C, var) in [(1, 2048, False), (16, 2048, False), (64, 2048, True), (128, 2021, True),
                            (256, 1024, False), (256, 2034, True), (512, 2034, True), (512, 4000, True)]:
            for (nq, nkv, d) in [(32, 4, 64), (32, 8, 128)]:
                print(json.dumps(bench_attn(B, C, nq, nkv, d, 1, var)), flush=True)
                for grid in (512, 1024):
                    for per_wg in (1, 2, 4):
                        print(json.dumps(bench_attn_wl(B, C, nq, nkv, d, grid, per_wg, var)), flush=True)
    if "decode" in what or "prefill" in what:
        eng = LLMEngine(a.model, device="cuda", kv_cache_gb=float(os.environ.get("MB_KV_GB", "40")),
                        max_num_seqs=int(os.environ.get("MB_MAX_SEQS", "256")))
        if "decode" in what:
            Bs = [int(x) for x in os.environ.get("MB_DECODE_B", "1,8,32,64,128,256").split(",")]
            Cs = [int(x) for x in os.environ.get("MB_DECODE_C", "512,2048").split(",")]
            mcs = [int(x) for x in os.environ.get("MB_MIN_CHUNKS", str(eng.ATTN_MIN_CHUNK)).split(",")]
            for B in Bs:
                for C in Cs:
                    for mc in mcs:
                        eng.ATTN_MIN_CHUNK = mc
                        print(json.dumps(dict(bench_decode(eng, B, C), min_chunk=mc,
                                              attn_ch=os.environ.get("DLLM_ATTN_CH", "1"),
                                              bt_prefetch=os.environ.get("DLLM_ATTN_BT_PREFETCH", "0"))), flush=True)
        if "prefill" in what:
            for B, L in ((1, 512), (8, 1024), (32, 2048)):
                print(json.dumps(bench_prefill(eng, B, L)), flush=True)
