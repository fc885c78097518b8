"""Probe: hipBLASLt default heuristic vs PyTorch TunableOp-selected solutions for the decode GEMMs
of TinyLlama-1.1B at decode buckets above the custom-kernel range (M > 256).

Times each GEMM inside a captured hipGraph (cold weights: the graph rotates over copies so the
weight matrix is not L2-resident between iterations, as in a real decode step).
Usage: python scripts/tunableop_probe.py [out.jsonl]
"""
import json
import os
import sys
import time

import torch

SHAPES = [(2560, 2048), (2048, 2048), (11264, 2048), (2048, 5632), (32000, 2048)]  # (N, K)
MS = [int(x) for x in os.environ.get("PROBE_MS", "256,320,384,448,512").split(",")]


def bench(M, N, K, reps=20):
    dev = "cuda"
    copies = max(2, int(512 * 2**20 // (N * K * 2)))
    ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) for _ in range(min(copies, 8))]
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    for w in ws:
        torch.matmul(x, w.t(), out=out)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            for w in ws:
                torch.matmul(x, w.t(), out=out)
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) * 1e6 / (reps * len(ws))
    return us


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    tun = torch.cuda.tunable
    mode = os.environ.get("PROBE_MODE", "default")
    if mode == "tuned":
        tun.enable(True)
        tun.tuning_enable(True)
        tun.set_max_tuning_duration(int(os.environ.get("PROBE_TUNE_MS", "30")))
        if os.environ.get("PROBE_TUNE_FILE"):
            tun.set_filename(os.environ["PROBE_TUNE_FILE"])
    rows = []
    for M in MS:
        for N, K in SHAPES:
            if mode == "tuned":
                x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
                w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
                t0 = time.perf_counter()
                torch.matmul(x, w.t())
                torch.cuda.synchronize()
                tune_s = time.perf_counter() - t0
                tun.tuning_enable(False)
            else:
                tune_s = 0.0
            us = bench(M, N, K)
            if mode == "tuned":
                tun.tuning_enable(True)
            tf = 2.0 * M * N * K / us / 1e6
            gbs = (N * K * 2 + M * K * 2 + M * N * 2) / us / 1e3
            r = dict(mode=mode, M=M, N=N, K=K, us=round(us, 2), tflops=round(tf, 1), gbs=round(gbs, 1),
                     tune_s=round(tune_s, 2))
            print(json.dumps(r), flush=True)
            rows.append(r)
    if mode == "tuned" and hasattr(tun, "write_file"):
        tun.write_file()
    if out:
        with open(out, "a") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
