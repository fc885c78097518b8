"""Run ONE tgemm plan (or hipBLASLt: plan "blas") on one shape a few times (for rocprofv3 --pmc passes).
Usage: python scripts/exp/tg_one.py M N K bm,bn,stages,splits,ks,waves[,k-groups,nl,sk,kdepth]|blas [reps]"""
import sys

import torch

from distributed_llm_amd.ops import gemm as G


def main():
    M, N, K = (int(v) for v in sys.argv[1:4])
    plan = None if sys.argv[4] == "blas" else tuple(int(v) for v in sys.argv[4].split(","))
    reps = int(sys.argv[5]) if len(sys.argv) > 5 else 10
    dev = torch.device("cuda:0")
    ext = G._native(torch.empty(1, device=dev))
    x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
    y = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    for _ in range(reps):
        if plan is None:
            torch.matmul(x, w.t(), out=y)   # hipBLASLt
        else:
            G._tgemm(ext, x, w, G.EPI_PLAIN, plan, y=y)
    torch.cuda.synchronize()
    print("done", M, N, K, plan)


if __name__ == "__main__":
    main()
