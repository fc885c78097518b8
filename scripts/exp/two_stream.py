"""Do two half-batch decode streams overlap?  TinyLlama's per-layer projections (22 layers x
[qkv 2560x2048, wo 2048x2048, gate|up 11264x2048, down 2048x5632]) as one M=B graph on one stream vs
two M=B/2 chains on two streams inside one graph (fork/join).  Weights are distinct per layer."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from distributed_llm_amd.ops import gemm as G

dev = "cuda"
G.reserve(dev)
L = 22
shapes = [(2560, 2048), (2048, 2048), (11264, 2048), (2048, 5632)]
W = [[(torch.randn(n, k, device=dev) * 0.02).to(torch.bfloat16) for n, k in shapes] for _ in range(L)]


def chain(x_by_k, M):
    for l in range(L):
        for (n, k), w in zip(shapes, W[l]):
            G.linear(x_by_k[k][:M], w)


def timed(fn, iters=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


for B in (128, 256, 320, 512):
    xa = {k: torch.randn(B, k, device=dev).to(torch.bfloat16) for k in (2048, 5632)}
    xb = {k: torch.randn(B, k, device=dev).to(torch.bfloat16) for k in (2048, 5632)}
    G.autotune([(n, k, False) for n, k in shapes], [B, B // 2], dev)
    one = timed(lambda: chain(xa, B))

    def two():
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with G.workspace_owner("side"), torch.cuda.stream(side):
            chain(xb, B // 2)
        chain(xa, B // 2)
        torch.cuda.current_stream().wait_stream(side)
    G.reserve(dev)
    with G.workspace_owner("side"):
        G.reserve(dev)
    t2 = timed(two)
    half = timed(lambda: chain(xa, B // 2))
    print({"B": B, "one_stream_ms": round(one, 3), "two_streams_half_each_ms": round(t2, 3),
           "one_half_batch_ms": round(half, 3)}, flush=True)
