"""Routing-cache scorer at scale (csrc/kernels/cosine.hip cache_scan_kernel) on one MI355X.

The reference's semantic lookup is a per-entry Python loop over at most cache_max_size=500 entries
(src/cache.py:267-305); the SURVEY sizes the HBM table for 288 GB.  For N = 1e4 .. 1e8 rows of 384
f32 (1e8 rows = 154 GB) this times one launch of the batched scorer:
  * ``ctx8``: ~8 rows per context (rows of a context scattered over the table, as LRU slot reuse
    leaves them): a lookup reads 4 B of context id per row plus its own context's rows;
  * ``ctx1``: every row in ONE context - the old per-query kernel's bytes (it scanned every row's
    1.5 KB for every query): the bound a context-blind scorer pays.
Bytes counted = 4 N (context ids) + 1,536 x matching rows x (1 row fetch; queries are L2-resident).
Also the whole host path (EmbeddingIndex.best_batch: pybind descriptor, launch, one read-back).
Usage: python scripts/cache_scorer_bench.py [--max-rows 1e8] > gpurun_out/cache_scorer.jsonl
"""
import argparse
import os
import sys
import json
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_llm_amd import ops
from distributed_llm_amd.router.cache import EmbeddingIndex


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / reps   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-rows", type=float, default=1e8)
    ap.add_argument("--dim", type=int, default=384)
    a = ap.parse_args()
    dev = torch.device("cuda")
    d = a.dim
    for n in (10_000, 1_000_000, 10_000_000, 100_000_000):
        if n > a.max_rows:
            break
        table = torch.empty((n, d), dtype=torch.float32, device=dev)
        step = 1 << 22
        for i in range(0, n, step):
            table[i:i + step].normal_()
        r = torch.arange(n, device=dev, dtype=torch.int64)
        nctx = max(1, n // 8)
        ctx8 = ((r * 2654435761) % nctx).to(torch.int32)
        ctx1 = torch.zeros(n, dtype=torch.int32, device=dev)
        del r
        g = torch.Generator(device="cpu").manual_seed(0)
        for mode, ctx in (("ctx8", ctx8), ("ctx1", ctx1)):
            for B in (1, 64, 128):
                if mode == "ctx1" and B > 1 and n > 1_000_000:
                    continue   # B full-table dot products per row: VALU-bound, not a lookup shape
                qs = [torch.randn(d, device=dev) for _ in range(B)]
                if mode == "ctx8":
                    cids = [int(x) for x in torch.randint(0, nctx, (B,), generator=g)]
                    matched = sum(int((ctx8 == c).sum()) for c in set(cids))
                else:
                    cids = [0] * B
                    matched = n
                best = torch.empty(B, dtype=torch.int64, device=dev)
                ext = ops._native(table)
                ptrs = [q.data_ptr() for q in qs]
                reps = 20 if n * (1 if mode == "ctx8" else 384) < 4e9 else 3
                us = timed(lambda: ext.cache_scan(ptrs, cids, table, ctx, n, 0.5, best), reps)
                byts = 4 * n + d * 4 * matched
                rec = {"rows": n, "table_gb": round(n * d * 4 / 1e9, 2), "mode": mode, "queries": B,
                       "matched_rows": matched, "us": round(us, 1), "bytes": byts,
                       "tb_s": round(byts / us / 1e6, 2)}
                if mode == "ctx1" and B == 1:
                    rec["note"] = "every row matches: the context-blind scan's bytes"
                print(json.dumps(rec), flush=True)
        # the whole host path of a batch lookup through the index (no table copy: adopt the tensors)
        if n <= 10_000_000:
            idx = EmbeddingIndex(dim=d, capacity=8, device="cuda")
            idx.table, idx.ctx, idx.capacity, idx._next = table, ctx8, n, n
            keys = [f"c{i}" for i in range(128)]
            for i, k in enumerate(keys):
                idx._ctx_ids[k] = i
            for B in (1, 64):
                qs = [torch.randn(d, device=dev) for _ in range(B)]
                idx.best_batch(qs, keys[:B], 0.5)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(20):
                    idx.best_batch(qs, keys[:B], 0.5)
                wall = (time.perf_counter() - t0) / 20 * 1e6
                print(json.dumps({"rows": n, "mode": "host_path_best_batch", "queries": B,
                                  "us_per_batch": round(wall, 1), "us_per_lookup": round(wall / B, 2)}), flush=True)
        del table, ctx8, ctx1
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
