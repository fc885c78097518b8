"""Probe: does splitting a decode batch in two halves on two HIP streams overlap the bandwidth-bound
paged attention of one half with the MFMA-bound GEMMs of the other?

Flagship shape (TinyLlama: H 2048, nq 32, nkv 4, d 64, I 5632), batch B, contexts uniform in
[C/4, 7C/4].  Per "layer": QKV, Wo, gate|up, down GEMMs (ops.linear) + persistent work-list paged
attention.  Arms, each over L layers, event-timed:
  serial : one stream, batch B
  halves : one stream, two B/2 halves one after the other (the cost of halving alone)
  overlap: two streams, one B/2 half each, no cross-stream dependencies (the best case of a
           two-micro-batch decode step)
Prints JSON lines.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from distributed_llm_amd import ops  # noqa: E402

H, NQ, NKV, D, I = 2048, 32, 4, 64, 5632
BS = 16


class Half:
    """One micro-batch: its queries, block tables, work list and attention workspace."""

    def __init__(self, ctxs, kc, vc, free_blocks, grid):
        dev = "cuda"
        B = len(ctxs)
        self.B = B
        nb = max(-(-c // BS) for c in ctxs)
        take = free_blocks[:B * nb]
        del free_blocks[:B * nb]
        self.bt = torch.tensor(np.array(take, dtype=np.int32).reshape(B, nb), device=dev)
        lens = np.array(ctxs, dtype=np.int64)
        order = np.argsort(-lens, kind="stable")
        I32 = lambda x: torch.tensor(np.asarray(x, dtype=np.int32), device=dev)  # noqa: E731
        self.qstart, self.qlen, self.ctx = I32(np.arange(B)), I32(np.ones(B)), I32(lens)
        self.tseq, self.ttok = I32(order), I32(np.zeros(B))
        items = ops.decode_work_items(lens[order], NKV, 16, grid, min_chunk=256, seq=order, qstart=order)
        self.items = I32(items)
        self.grid = grid
        ws = B * NKV * 16 * 16
        self.wsp = (torch.empty(ws * D, dtype=torch.float32, device=dev),
                    torch.empty(ws * 2, dtype=torch.float32, device=dev),
                    torch.zeros(B * NKV + 2, dtype=torch.int32, device=dev))
        self.q = torch.randn(B, NQ, D, device=dev).to(torch.bfloat16)
        self.x = torch.randn(B, H, device=dev).to(torch.bfloat16)
        self.a = torch.randn(B, I, device=dev).to(torch.bfloat16)
        self.kc, self.vc = kc, vc

    def attn(self):
        return ops.paged_attention(self.q, self.kc, self.vc, self.bt, self.qstart, self.qlen, self.ctx, self.tseq,
                                   self.ttok, splits=16, workspace=self.wsp, items=self.items, grid_items=self.grid)

    def gemms(self, W):
        ops.linear(self.x, W["qkv"])
        ops.linear(self.x, W["wo"])
        ops.linear(self.x, W["gu"])
        ops.linear(self.a, W["wd"])

    def layer(self, W):
        self.gemms(W)
        self.attn()


def timed(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(iters):
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e))
    return best


def main():
    B = int(os.environ.get("B", 480))
    C = int(os.environ.get("C", 1400))
    L = int(os.environ.get("L", 22))
    g = np.random.default_rng(0)
    ctxs = g.integers(C // 4, 7 * C // 4 + 1, B).tolist()
    need = sum(-(-c // BS) for c in ctxs) * 2 + 64   # full batch + two halves, disjoint blocks
    nblk = need
    kc = torch.randn(nblk, NKV, BS, D, device="cuda").to(torch.bfloat16)
    vc = torch.randn(nblk, NKV, D, BS, device="cuda").to(torch.bfloat16)
    free = g.permutation(nblk).tolist()
    Ws = [{"qkv": torch.randn((NQ + 2 * NKV) * D, H, device="cuda").to(torch.bfloat16) * 0.02,
           "wo": torch.randn(H, NQ * D, device="cuda").to(torch.bfloat16) * 0.02,
           "gu": torch.randn(2 * I, H, device="cuda").to(torch.bfloat16) * 0.02,
           "wd": torch.randn(H, I, device="cuda").to(torch.bfloat16) * 0.02} for _ in range(L)]
    for grid_full, grid_half in ((512, 256), (512, 512)):
        full = Half(ctxs, kc, vc, list(free), grid_full)
        rest = list(free)
        h0 = Half(ctxs[0::2], kc, vc, rest, grid_half)
        h1 = Half(ctxs[1::2], kc, vc, rest, grid_half)
        s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
        cur = torch.cuda.current_stream()

        def serial():
            for W in Ws:
                full.layer(W)

        def halves():
            for W in Ws:
                h0.layer(W)
                h1.layer(W)

        def overlap():
            s0.wait_stream(cur)
            s1.wait_stream(cur)
            with torch.cuda.stream(s0):
                for W in Ws:
                    h0.layer(W)
            with torch.cuda.stream(s1):
                for W in Ws:
                    h1.layer(W)
            cur.wait_stream(s0)
            cur.wait_stream(s1)

        def attn_only():
            for _ in Ws:
                full.attn()

        def gemm_only():
            for W in Ws:
                full.gemms(W)

        def attn_half_only():
            for _ in Ws:
                h0.attn()

        def gemm_half_only():
            for W in Ws:
                h0.gemms(W)

        res = {"B": B, "C": C, "L": L, "grid_full": grid_full, "grid_half": grid_half}
        for name, fn in (("attn_only", attn_only), ("gemm_only", gemm_only), ("attn_half", attn_half_only),
                         ("gemm_half", gemm_half_only), ("serial", serial), ("halves", halves),
                         ("overlap", overlap)):
            res[name + "_ms"] = round(timed(fn), 3)
            print(json.dumps({"arm": name, "ms": res[name + "_ms"]}), flush=True)
        res["overlap_vs_serial"] = round(res["overlap_ms"] / res["serial_ms"], 3)
        print(json.dumps(res), flush=True)
        # numerics of the overlapped halves: same outputs as the halves run alone
        o_a = h0.attn().float()
        torch.cuda.synchronize()
        overlap()
        torch.cuda.synchronize()
        o_b = h0.attn().float()
        print(json.dumps({"attn_repeatable": bool(torch.equal(o_a, o_b))}), flush=True)


if __name__ == "__main__":
    main()
