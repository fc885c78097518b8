"""32-deep k-step tgemm plans (GemmArgs.kdepth = 32: 256-row tiles with 4-6 stage rings) against
hipBLASLt (+ the standalone epilogue a fused op then needs) and the best 64-deep tgemm plans, at
decode (M = 512) and prefill (M = 2048-8192) sizes; row-major and K-panel weights.  One JSON line
per (shape, M); hipGraph replays over rotated weights (ops.gemm._time); max relative error of each
k32 plan against F.linear."""
import json
import sys

import torch
import torch.nn.functional as F

from distributed_llm_amd.ops import gemm as G

SHAPES = {"tinyllama": [(2560, 2048), (2048, 2048), (11264, 2048), (2048, 5632)],
          "llama3-8b": [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]}
K64 = [(256, 128, 3, 1, 1, 8, 1, 8), (256, 256, 2, 1, 1, 8), (128, 128, 3, 1, 1, 8), (64, 128, 3, 1, 2, 8),
       (128, 64, 4, 1, 1, 4, 1, 8), (64, 64, 4, 1, 1, 4, 1, 8)]
K32 = [(bm, bn, st, 1, 1, 8, 1, nl, 0, 32) for bm, bn, st, nl in G._TG_K32]


def main():
    dev = torch.device("cuda:0")
    ms = [int(a) for a in sys.argv[1:]] or [512, 2048, 4096, 8192]
    ext = G._native(torch.empty(1, device=dev))
    for fam, shapes in SHAPES.items():
        for N, K in shapes:
            copies = max(2, min(16, (512 << 20) // (N * K * 2)))
            ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(copies)]
            wps = [G.panel_weight(w) for w in ws]
            for M in ms:
                x = torch.randn(M, K, device=dev).to(torch.bfloat16)
                y = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
                flops = 2.0 * M * N * K
                res = {"blas": G._time(lambda i: torch.matmul(x, ws[i % copies].t(), out=y), iters=8)}
                res["post"] = G._post_us(M, N, dev)
                ref = F.linear(x, ws[0]).float()
                errs = {}
                for p in K64 + K32:
                    for tag, wl in (("row", ws), ("pan", wps)):
                        key = f"{tag}{p[:4]}{'k32' if len(p) > 9 else ''}w{p[5]}nl{p[7] if len(p) > 7 else 0}"
                        try:
                            res[key] = G._time(lambda i: G._tgemm(ext, x, wl[i % copies], G.EPI_PLAIN, p, y=y), iters=8)
                        except Exception:  # noqa: BLE001 - plan refused for this shape
                            res[key] = None
                            continue
                        if len(p) > 9:
                            y.zero_()
                            G._tgemm(ext, x, wl[0], G.EPI_PLAIN, p, y=y)
                            errs[key] = round(float((y.float() - ref).abs().max() / ref.abs().max()), 5)
                k32 = {k: v for k, v in res.items() if "k32" in k and v}
                k64 = {k: v for k, v in res.items() if k.startswith(("row", "pan")) and "k32" not in k and v}
                b32 = min(k32.items(), key=lambda kv: kv[1]) if k32 else (None, None)
                b64 = min(k64.items(), key=lambda kv: kv[1]) if k64 else (None, None)
                print(json.dumps({"fam": fam, "M": M, "N": N, "K": K, "blas_us": round(res["blas"], 1),
                                  "blas_post_us": round(res["blas"] + res["post"], 1),
                                  "best_k32": b32[0], "k32_us": b32[1] and round(b32[1], 1),
                                  "best_k64": b64[0], "k64_us": b64[1] and round(b64[1], 1),
                                  "blas_tf": round(flops / res["blas"] / 1e6),
                                  "k32_tf": b32[1] and round(flops / b32[1] / 1e6), "k32_err": errs,
                                  "all": {k: (round(v, 1) if v else None) for k, v in res.items()}}), flush=True)
            del ws, wps


if __name__ == "__main__":
    main()
