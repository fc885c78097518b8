"""Grouped tile raster for tgemm (GemmArgs.raster): the 256-row tiles at prefill and decode sizes
with raster 0 (n-major) and groups of 2 / 4 / 8 m-tiles, against hipBLASLt (PLAIN epilogue,
hipGraph replays over rotated weight copies).
Usage: python scripts/exp/raster_probe.py > gpurun_out/raster_probe.jsonl"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from distributed_llm_amd.ops import gemm as G  # noqa: E402

SHAPES = [(480, 11264, 2048), (2048, 11264, 2048), (4096, 2048, 5632), (8192, 11264, 2048), (4096, 4096, 14336),
          (4096, 6144, 4096), (2048, 28672, 4096), (2048, 4096, 4096)]
PLANS = [(256, 256, 2, 1, 1, 8, 1, 0, 0, 64, 16), (256, 256, 4, 1, 1, 8, 1, 0, 0, 32, 16),
         (256, 128, 3, 1, 1, 8, 1, 8, 0, 64, 16), (256, 128, 3, 1, 1, 8, 1, 0, 0, 64, 16)]


def main():
    dev = torch.device("cuda")
    G.reserve(dev)
    ext = G._native(torch.empty(1, device=dev))
    for (M, N, K) in SHAPES:
        copies = max(2, min(16, (512 << 20) // (N * K * 2)))
        ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(copies)]
        wps = [G.panel_weight(w) for w in ws]
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        y = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        out = {"M": M, "N": N, "K": K,
               "blas_us": round(G._time(lambda i: torch.matmul(x, ws[i % copies].t(), out=y), iters=8), 2)}
        for p in PLANS:
            for r in (0, 2, 4, 8):
                plan = p + (r,)
                try:
                    t = G._time(lambda i: G._tgemm(ext, x, wps[i % copies], G.EPI_PLAIN, plan, y=y), iters=8)
                except Exception:  # noqa: BLE001
                    t = None
                out["%dx%d st%d k%d nl%d r%d" % (p[0], p[1], p[2], p[9], p[7], r)] = round(t, 2) if t else None
        print(json.dumps(out), flush=True)
        del ws, wps, x, y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
