"""Do two decode-step graphs overlap on one MI355X?  (feasibility probe for nano-batching)

Two engines (separate buffers and weights, TinyLlama) each fabricate a half batch (B/2 rows at
context C) and capture their decode graph.  Times, per step:
  full       : one engine's graph at the full batch B
  serial     : half-batch graph A then graph B on one stream
  concurrent : graph A on stream 1 and graph B on stream 2 (fork/join once per step)
A concurrent time well below serial would mean the memory-bound attention of one half-batch and
the GEMMs of the other share the GPU; near serial means they do not.
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(__file__), "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
from distributed_llm_amd import ops  # noqa: E402
from distributed_llm_amd.engine.llm_engine import LLMEngine  # noqa: E402


def prepare(eng, B, C, base):
    bm = eng.bm
    rows = []
    for i in range(B):
        sid = base + i
        tbl, _ = bm.allocate(sid, [5 + (i % 1000)] + [5] * (C - 1))
        assert tbl, "KV cache too small"
        row = eng._free_rows.pop()
        t = bm.block_table(sid)
        eng.bt_host[row, :len(t)] = t
        rows.append(row)
    eng._bt_dirty = True
    bs = eng._bucket(B)
    o, h, R = eng._off, eng.dec_host, eng.R
    rows = np.array(rows)
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
    eng._sync_bt()
    eng.dec_dev.copy_(eng.dec_host_t)
    if eng._use_worklist(bs):
        items_t, items = eng._items_bufs[0]
        ops.decode_work_items(np.full(B, C), eng.model.nkv, eng.max_splits,
                              eng.ATTN_ITEMS_PER_WG * eng._attn_grid(bs), min_chunk=eng.ATTN_MIN_CHUNK, out=items,
                              seq=rows, qstart=np.arange(B))
        n = ops.work_items_len(items)
        eng.items_dev[:n].copy_(items_t[:n])
    return eng._graphs.get(eng._gkey(bs, 0)) or eng._capture(bs, 0)


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) * 1000 / iters


def main():
    B = int(os.environ.get("PROBE_B", "512"))
    C = int(os.environ.get("PROBE_C", "2048"))
    kw = dict(device="cuda", kv_cache_gb=float(os.environ.get("PROBE_KV_GB", "48")), max_num_seqs=B)
    ea = LLMEngine("tinyllama-1.1b", **kw)
    eb = LLMEngine("tinyllama-1.1b", seed=1, **kw)
    gfull = prepare(ea, B, C, 10_000_000)
    full = timed(gfull.replay)
    for s_ in range(B):
        ea.bm.free(10_000_000 + s_)
    ea._free_rows = list(range(ea.R))
    ea.bt_host[:] = 0
    ga = prepare(ea, B // 2, C, 20_000_000)
    gb = prepare(eb, B // 2, C, 30_000_000)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def serial():
        ga.replay()
        gb.replay()

    def concurrent():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            ga.replay()
        with torch.cuda.stream(s2):
            gb.replay()
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    ser = timed(serial)
    con = timed(concurrent)
    print(json.dumps({"B": B, "C": C, "full_ms": round(full, 3), "serial_halves_ms": round(ser, 3),
                      "concurrent_halves_ms": round(con, 3), "concurrent_vs_full": round(full / con, 3)}), flush=True)


if __name__ == "__main__":
    main()
