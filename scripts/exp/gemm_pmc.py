"""PMC probe of one decode-size GEMM (run under rocprofv3 --pmc): tgemm plan vs hipBLASLt on the
same shape, 200 eager launches each over rotated weight copies (weights stream from HBM)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import torch.nn.functional as F

from distributed_llm_amd import ops
from distributed_llm_amd.ops import gemm as G

M, N, K = (int(v) for v in os.environ.get("PMC_SHAPE", "320,2048,2048").split(","))
plan = tuple(int(v) for v in os.environ.get("PMC_PLAN", "64,64,3,1,2,4").split(","))
G.reserve("cuda")
copies = 32
ws = [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(copies)]
x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
ext = ops._native(x)
for i in range(200):
    G._tgemm(ext, x, ws[i % copies], G.EPI_PLAIN, plan, y=y)
torch.cuda.synchronize()
for i in range(200):
    F.linear(x, ws[i % copies])
torch.cuda.synchronize()
print("done", M, N, K, plan)
