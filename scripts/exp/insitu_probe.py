"""Fused-op core options of TinyLlama's decoder layer at the flagship's decode buckets, timed both
ways: the stand-ins (PLAIN tgemm, RESADD GEMV / skinny_epi) and in situ (ops.gemm._retime_fused).
Usage: python scripts/exp/insitu_probe.py [M ...]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from distributed_llm_amd.ops import gemm as G  # noqa: E402

H, I, NQ, NKV, D = 2048, 5632, 32, 4, 64
FUSED = [((NQ + 2 * NKV) * D, H), (H, NQ * D), (2 * I, H), (H, I)]


def main():
    ms = [int(a) for a in sys.argv[1:]] or [448, 512]
    shapes = sorted({(n, k, False) for n, k in FUSED})
    for insitu in (False, True):
        G.FUSED_INSITU = insitu
        G._P.fused_core.clear(); G._P.fused_opts.clear(); G._P.tg_plans.clear(); G._P.plans.clear()
        G.autotune(shapes, ms, "cuda", verbose=False, fused=FUSED, qkv_dims=(NQ, NKV, D))
        for M in ms:
            for n, k in FUSED:
                opts = G._P.fused_opts[(M, n, k)]
                print(("in-situ " if insitu else "stand-in"), M, n, k, G._P.fused_core[(M, n, k)],
                      " ".join(f"{c}:{t:.1f}" for c, t in sorted(opts.items(), key=lambda kv: kv[1])), flush=True)


if __name__ == "__main__":
    main()
