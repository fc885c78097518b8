"""Batch-1..8 decode GEMV (csrc/kernels/gemv.hip) against the streaming-read floor
(scripts/exp/streamfloor.hip): each projection of TinyLlama and Llama-3-8B timed PLAIN and with its
fused epilogue (RESADD / QKV / SWIGLU), R = 1, 2, 4, hipGraph replays over rotated weights
(ops.gemm._time), one JSON line per (model, projection, M, grid policy).  DLLM_GEMV_GRIDS =
"min:xdiv:nmin,..." A/Bs the batch 2-8 grid policies (gemv.hip gemv_grid; xdiv 0 = one workgroup per
column block) in one process."""
import os
import json
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from distributed_llm_amd import ops  # noqa: E402
from distributed_llm_amd.ops import gemm as G  # noqa: E402

MODELS = {
    "tinyllama": dict(H=2048, NQ=32, NKV=4, D=64, I=5632, V=32000),
    "llama3-8b": dict(H=4096, NQ=32, NKV=8, D=128, I=14336, V=128256),
}


def main():
    dev = torch.device("cuda:0")
    ms = [int(a) for a in sys.argv[1:]] or [1]
    ext = G._native(torch.empty(1, device=dev))
    grids = [tuple(int(v) for v in g.split(":")) for g in os.environ.get("DLLM_GEMV_GRIDS", "512:4:8192").split(",")]
    for name, c in MODELS.items():
        H, NQ, NKV, D, I = c["H"], c["NQ"], c["NKV"], c["D"], c["I"]
        shapes = {"qkv": ((NQ + 2 * NKV) * D, H), "wo": (H, NQ * D), "gate_up": (2 * I, H), "down": (H, I),
                  "lm_head": (c["V"], H)}
        blocks = 4096
        kc = torch.zeros(blocks, NKV, 16, D, dtype=torch.bfloat16, device=dev)
        vc = torch.zeros(blocks, NKV, D, 16, dtype=torch.bfloat16, device=dev)
        cs = ops.rope_cos_sin(4096, D, 10000.0, dev)
        for proj, (N, K) in shapes.items():
            copies = max(2, min(24, (3 << 30) // (N * K * 2)))
            ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(copies)]
            for M, grid in [(M, g) for M in ms for g in (grids if M > 1 else grids[:1])]:
                ext.gemv_set_grid(*grid)
                x = torch.randn(M, K, device=dev).to(torch.bfloat16)
                y = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
                row = {"model": name, "proj": proj, "M": M, "N": N, "K": K, "MB": round(N * K * 2 / 2**20, 1),
                       "grid": ":".join(map(str, grid))}
                for R in (1, 2, 4):
                    try:
                        row["plain_R%d" % R] = G._time(lambda i: ext.gemv(x, ws[i % copies], y, R, False), 24)
                        if proj == "lm_head":
                            pass
                        elif proj in ("wo", "down"):
                            res = torch.randn(M, N, device=dev).to(torch.bfloat16)
                            ssq = torch.empty(G.max_slots(N, M), M, dtype=torch.float32, device=dev)
                            row["resadd_R%d" % R] = G._time(lambda i: ext.gemv_resadd(x, ws[i % copies], res, ssq, R), 24)
                        elif proj == "gate_up":
                            ssq = torch.rand(512, M, device=dev) + 1.0
                            act = torch.empty(M, I, dtype=torch.bfloat16, device=dev)
                            row["swiglu_R%d" % R] = G._time(lambda i: ext.gemv_swiglu(x, ws[i % copies], ssq, 512, 1.0 / H,
                                                                                      1e-5, act, R), 24)
                        else:
                            ssq = torch.rand(512, M, device=dev) + 1.0
                            pos = torch.randint(0, 4000, (M,), dtype=torch.int32, device=dev)
                            slots = (torch.randperm(blocks * 16, device=dev)[:M]).to(torch.int32)
                            q = torch.empty(M, NQ, D, dtype=torch.bfloat16, device=dev)
                            row["qkv_R%d" % R] = G._time(lambda i: ext.gemv_qkv(x, ws[i % copies], ssq, 512, 1.0 / H, 1e-5,
                                                                                pos, cs, slots, q, kc, vc, NQ, NKV, D, R), 24)
                    except Exception as e:  # noqa: BLE001
                        row["error_R%d" % R] = str(e)[:120]
                print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in row.items()}), flush=True)
            del ws
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
