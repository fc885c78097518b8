"""Probe: cost of surplus (early-exit) split blocks in the dynamic split-K attention path."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_llm_amd import ops  # noqa: E402
from scripts.microbench import timeit  # noqa: E402


def main():
    B, C, nq, nkv, d = 256, 2000, 32, 8, 128
    g = torch.Generator().manual_seed(0)
    ctxs = torch.randint(C // 4, 7 * C // 4 + 1, (B,), generator=g).tolist()
    Cm = max(ctxs)
    NB = B * ((Cm + 15) // 16) + 8
    kc = torch.randn(NB, nkv, 16, d, device="cuda").to(torch.bfloat16)
    vc = torch.randn(NB, nkv, d, 16, device="cuda").to(torch.bfloat16)
    nb = (Cm + 15) // 16
    bt = torch.randperm(NB - 8, device="cuda")[:B * nb].view(B, nb).to(torch.int32)
    q = torch.randn(B, nq, d, device="cuda").to(torch.bfloat16)
    I = lambda x: torch.tensor(x, dtype=torch.int32, device="cuda")  # noqa: E731
    qs, ql, cx = I(list(range(B))), I([1] * B), I(ctxs)
    ts, tt = ops.build_tiles([1] * B, nq // nkv)
    ts, tt = I(ts), I(tt)
    nt = ts.numel()
    order = sorted(range(B), key=lambda i: -ctxs[i])
    ts_sorted = I([order[i] for i in range(B)]) if nq // nkv >= 1 else ts
    for name, tsx in (("unsorted", ts), ("longest_first", ts_sorted)):
        us = timeit(lambda: ops.paged_attention(q, kc, vc, bt, qs, ql, cx, tsx, tt, splits=1), iters=30) * 1000
        print(json.dumps({"z": 1, "order": name, "us": round(us, 1)}), flush=True)
    for z in (1, 2, 4, 8):
        ws = (torch.empty(nt * nkv * z * 16 * d, device="cuda"), torch.empty(nt * nkv * z * 16 * 2, device="cuda"),
              torch.zeros(nt * nkv, dtype=torch.int32, device="cuda"))
        for sl in (1 << 20, 2048, 1024, 512):
            slt = I([sl])
            us = timeit(lambda: ops.paged_attention(q, kc, vc, bt, qs, ql, cx, ts, tt, splits=z, workspace=ws,
                                                    split_len=slt if z > 1 else None), iters=30) * 1000
            print(json.dumps({"z": z, "split_len": sl, "us": round(us, 1)}), flush=True)
            if z == 1:
                break
        if z > 1:
            us = timeit(lambda: ops.paged_attention(q, kc, vc, bt, qs, ql, cx, ts, tt, splits=z, workspace=ws),
                        iters=30) * 1000
            print(json.dumps({"z": z, "split_len": "static", "us": round(us, 1)}), flush=True)


if __name__ == "__main__":
    main()
