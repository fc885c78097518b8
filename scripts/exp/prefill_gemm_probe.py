"""Prefill-size GEMMs (M = 2048-8192): hipBLASLt core (+ the standalone epilogue a fused op then
needs) against tgemm plans with the epilogue fused (PLAIN timed: the fused epilogues cost the
same pass over the output tile).  One JSON line per (shape, candidate); hipGraph replays over
rotated weights (ops.gemm._time)."""
import json
import sys

import torch
import torch.nn.functional as F

from distributed_llm_amd.ops import gemm as G

SHAPES = {"tinyllama": [(2560, 2048), (2048, 2048), (11264, 2048), (2048, 5632)],
          "llama3-8b": [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]}
PLANS = [(256, 256, 2, 1, 1, 8), (256, 256, 3, 1, 1, 8), (256, 128, 3, 1, 1, 8), (256, 128, 2, 1, 1, 8),
         (192, 128, 3, 1, 1, 8), (128, 128, 3, 1, 1, 8), (128, 128, 3, 1, 1, 4), (128, 128, 2, 1, 2, 4)]
PLANS = [p for p in PLANS if G.tg_built(p)]   # (pruned plans are not built: profiles/r6_prune.md)


def main():
    dev = torch.device("cuda:0")
    ms = [int(a) for a in sys.argv[1:]] or [2048, 4096, 8192]
    for fam, shapes in SHAPES.items():
        for N, K in shapes:
            copies = max(2, min(16, (512 << 20) // (N * K * 2)))
            ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(copies)]
            for M in ms:
                x = torch.randn(M, K, device=dev).to(torch.bfloat16)
                y = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
                flops = 2.0 * M * N * K
                res = {"blas": G._time(lambda i: torch.matmul(x, ws[i % copies].t(), out=y), iters=8)}
                res["post"] = G._post_us(M, N, dev)
                ext = G._native(x)
                wps = [G.panel_weight(w) for w in ws]   # the K-panel-major copies the fused decoder weights keep
                for p in PLANS:
                    for tag, wl in (("tg", ws), ("tgP", wps)):
                        try:
                            res[tag + str(p)] = G._time(lambda i: G._tgemm(ext, x, wl[i % copies], G.EPI_PLAIN, p, y=y),
                                                        iters=8)
                        except Exception as e:  # noqa: BLE001 - plan refused for this shape
                            res[tag + str(p)] = None
                del wps
                ref = F.linear(x, ws[0]).float()
                G._tgemm(ext, x, ws[0], G.EPI_PLAIN, PLANS[0], y=y)
                err = float((y.float() - ref).abs().max() / ref.abs().max())
                best_tg = min((v, k) for k, v in res.items() if k.startswith("tg") and v)
                best_row = min((v, k) for k, v in res.items() if k.startswith("tg(") and v)
                print(json.dumps({"fam": fam, "M": M, "N": N, "K": K, "blas_us": round(res["blas"], 1),
                                  "post_us": round(res["post"], 1), "best_tg": best_tg[1], "tg_us": round(best_tg[0], 1),
                                  "best_rowmajor_us": round(best_row[0], 1),
                                  "blas_tf": round(flops / res["blas"] / 1e6), "tg_tf": round(flops / best_tg[0] / 1e6),
                                  "err_256": err, "all": {k: (round(v, 1) if v else None) for k, v in res.items()}}),
                      flush=True)
            del ws


if __name__ == "__main__":
    main()
