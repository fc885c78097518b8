"""Decode-GEMM library probe: hipBLASLt vs rocBLAS vs TunableOp for the flagship's per-layer
shapes at decode batch sizes, weights rotated through > MALL capacity (cold like in a real step),
timed over hipGraph-captured loops (no launch gaps).  Prints JSON lines."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

SHAPES = [(2560, 2048), (2048, 2048), (11264, 2048), (2048, 5632)]


def run(lib, Ms):
    if lib != "default":
        torch.backends.cuda.preferred_blas_library(lib)
    out = []
    for (N, K) in SHAPES:
        copies = max(2, (768 << 20) // (N * K * 2))
        ws = [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(copies)]
        for M in Ms:
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            for w in ws[:2]:
                F.linear(x, w)  # warm-up / tuning outside capture
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for w in ws:
                    F.linear(x, w)
            torch.cuda.current_stream().wait_stream(s)
            with torch.cuda.graph(g):
                for w in ws:
                    F.linear(x, w)
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1000 / (5 * copies)
            r = {"lib": lib, "M": M, "N": N, "K": K, "us": round(us, 2),
                 "weight_TBps": round(N * K * 2 / us / 1e6, 2), "TFLOPs": round(2 * M * N * K / us / 1e6, 1)}
            print(json.dumps(r), flush=True)
            out.append(r)
        del ws
    return out


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else "default"
    run(lib, [64, 128, 256])
