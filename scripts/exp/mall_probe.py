"""Infinity-Cache (MALL) probe for single-stream decode GEMVs (1x MI355X).

Times the batch-1 GEMV of each TinyLlama / Llama-3-8B projection (graph of 24 calls) with
  cold : 24 rotated weight copies (every call streams from HBM, as in decode),
  hot  : one weight (after the first call it is resident in the 256 MiB Infinity Cache),
Prints one JSON line per shape.  Measured (profiles/r2_decode_gemm_floors.md): hot saves only the
~1.3 us of the first HBM round trip; a layer-ahead prefetch kernel on a forked graph branch cost
more than that in fork/join (the prefetch variant was removed after the measurement).
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from distributed_llm_amd import ops  # noqa: E402


def graph_time(fn, iters=24):
    fn(0)
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


def main():
    ext = ops._native(torch.empty(1, device="cuda"))
    for (N, K) in [(2560, 2048), (2048, 2048), (11264, 2048), (2048, 5632), (6144, 4096), (28672, 4096),
                   (4096, 14336)]:
        copies = 24
        ws = [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(copies)]
        x = torch.randn(1, K, device="cuda").to(torch.bfloat16)
        y = torch.empty(1, N, dtype=torch.bfloat16, device="cuda")
        cold = graph_time(lambda i: ext.gemv(x, ws[i % copies], y, 1, False))
        hot = graph_time(lambda i: ext.gemv(x, ws[0], y, 1, False))
        mb = N * K * 2 / 1e6
        print(json.dumps({"N": N, "K": K, "MB": round(mb, 1), "cold_us": round(cold, 2), "hot_us": round(hot, 2),
                          "cold_TBps": round(mb / cold, 2), "hot_TBps": round(mb / hot, 2)}), flush=True)
        del ws


if __name__ == "__main__":
    main()
