"""32 x 32 x 16 MFMA tgemm plans (tgemm.hip by_tile_m32) against their 16 x 16 x 32 twins and
hipBLASLt on the flagship's decode shapes (TinyLlama, M = 480) and prefill shapes (PLAIN
epilogue; hipGraph replays over rotated weight copies, as ops.gemm autotunes).
Usage: python scripts/exp/m32_probe.py > gpurun_out/m32_probe.jsonl"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from distributed_llm_amd.ops import gemm as G  # noqa: E402

DECODE = [(480, 2560, 2048), (480, 2048, 2048), (480, 11264, 2048), (480, 2048, 5632)]
PREFILL = [(2048, 11264, 2048), (4096, 4096, 14336), (4096, 6144, 4096), (2048, 28672, 4096)]
PAIRS16 = [(64, 64, 3, 1, 2, 4), (64, 128, 3, 1, 2, 8), (128, 64, 4, 1, 1, 4, 1, 8), (256, 128, 3, 1, 1, 8, 1, 8),
           (256, 256, 2, 1, 1, 8)]


def main():
    dev = torch.device("cuda")
    G.reserve(dev)
    ext = G._native(torch.empty(1, device=dev))
    for (M, N, K) in DECODE + PREFILL:
        copies = max(2, min(16, (512 << 20) // (N * K * 2)))
        ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(copies)]
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        y = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        res = {"blas": G._time(lambda i: torch.matmul(x, ws[i % copies].t(), out=y), iters=8)}
        for p16 in PAIRS16:
            for sp in ((1, 2, 3, 4) if M < 1024 else (1,)):
                base = p16[:3] + (sp,) + p16[4:]
                p16f = tuple(base) + ((1, 0, 0, 64) if len(base) == 6 else (0, 64)) + (16,)
                p32 = p16f[:10] + (32,)
                for tag, p in (("m16", p16f), ("m32", p32)):
                    try:
                        t = G._time(lambda i: G._tgemm(ext, x, ws[i % copies], G.EPI_PLAIN, p, y=y), iters=8)
                    except Exception as e:  # noqa: BLE001 - plan refused (workspace, shape)
                        t = None
                    res[f"{tag}:{p[:4]}"] = t
        best16 = min((v, k) for k, v in res.items() if k.startswith("m16") and v)
        best32 = min((v, k) for k, v in res.items() if k.startswith("m32") and v)
        print(json.dumps({"M": M, "N": N, "K": K, "blas_us": round(res["blas"], 2),
                          "best_m16": [best16[1], round(best16[0], 2)], "best_m32": [best32[1], round(best32[0], 2)],
                          "m32_over_m16": round(best32[0] / best16[0], 3),
                          "tflops_m32": round(2 * M * N * K / best32[0] / 1e6, 1),
                          "all": {k: (round(v, 2) if v else None) for k, v in res.items()}}), flush=True)
        del ws, x, y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
