"""Cost of the fused decoder epilogues at decode batch sizes: the same tgemm plan timed PLAIN and
with the QKV (RoPE + q out + paged K / V^T writes), RESADD (in-place residual + row sums) and
SwiGLU epilogues, TinyLlama shapes, hipGraph replays over rotated weights (ops.gemm._time)."""
import json
import sys

import torch

from distributed_llm_amd import ops
from distributed_llm_amd.ops import gemm as G

H, NQ, NKV, D, I = 2048, 32, 4, 64, 5632
PLANS = [(64, 64, 4, 1, 1, 4), (64, 64, 4, 1, 1, 4, 1, 8), (64, 128, 3, 1, 1, 8)]


def main():
    dev = torch.device("cuda:0")
    ms = [int(a) for a in sys.argv[1:]] or [320, 512]
    nq_cols = (NQ + 2 * NKV) * D
    copies = 8
    wq = [(torch.randn(nq_cols, H, device=dev) * 0.02).to(torch.bfloat16) for _ in range(copies)]
    wo = [(torch.randn(H, NQ * D, device=dev) * 0.02).to(torch.bfloat16) for _ in range(copies)]
    wgu = [(torch.randn(2 * I, H, device=dev) * 0.02).to(torch.bfloat16) for _ in range(copies)]
    blocks = 8192
    kc = torch.zeros(blocks, NKV, 16, D, dtype=torch.bfloat16, device=dev)
    vc = torch.zeros(blocks, NKV, D, 16, dtype=torch.bfloat16, device=dev)
    cs = ops.rope_cos_sin(4096, D, 10000.0, dev)
    for M in ms:
        ext = G._native(torch.empty(1, device=dev))
        r = torch.randn(M, H, device=dev).to(torch.bfloat16)
        o = torch.randn(M, NQ * D, device=dev).to(torch.bfloat16)
        y = torch.empty(M, max(nq_cols, 2 * I), dtype=torch.bfloat16, device=dev)
        ssq = torch.rand(64, M, device=dev) + 1.0
        pos = torch.randint(0, 4000, (M,), dtype=torch.int32, device=dev)
        slots = (torch.randperm(blocks * 16, device=dev)[:M]).to(torch.int32)
        q = torch.empty(M, NQ, D, dtype=torch.bfloat16, device=dev)
        act = torch.empty(M, I, dtype=torch.bfloat16, device=dev)
        for p in PLANS:
            row = {"M": M, "plan": p}
            try:
                row["qkv_plain"] = G._time(lambda i: G._tgemm(ext, r, wq[i % copies], G.EPI_PLAIN, p, y=y[:, :nq_cols]), 16)
                row["qkv_epi"] = G._time(lambda i: G._tgemm(ext, r, wq[i % copies], G.EPI_QKV, p, ssq_in=ssq, ssq_n=8,
                                                            norm_scale=1.0 / H, eps=1e-5, pos=pos, cos_sin=cs, slots=slots,
                                                            q_out=q, kc=kc, vc=vc, nq=NQ, nkv=NKV, d=D), 16)
                noslot = torch.full_like(slots, -1)      # K / V cache writes skipped: RoPE + q only
                row["qkv_epi_q_only"] = G._time(lambda i: G._tgemm(ext, r, wq[i % copies], G.EPI_QKV, p, ssq_in=ssq, ssq_n=8,
                                                                   norm_scale=1.0 / H, eps=1e-5, pos=pos, cos_sin=cs,
                                                                   slots=noslot, q_out=q, kc=kc, vc=vc, nq=NQ, nkv=NKV,
                                                                   d=D), 16)
                seq = torch.arange(M, dtype=torch.int32, device=dev) * 16   # one row per block, offset 0
                row["qkv_epi_seq_slots"] = G._time(lambda i: G._tgemm(ext, r, wq[i % copies], G.EPI_QKV, p, ssq_in=ssq,
                                                                      ssq_n=8, norm_scale=1.0 / H, eps=1e-5, pos=pos,
                                                                      cos_sin=cs, slots=seq, q_out=q, kc=kc, vc=vc, nq=NQ,
                                                                      nkv=NKV, d=D), 16)
                row["qkv_plain_rowscale"] = G._time(lambda i: G._tgemm(ext, r, wq[i % copies], G.EPI_PLAIN, p,
                                                                       y=y[:, :nq_cols], ssq_in=ssq, ssq_n=8,
                                                                       norm_scale=1.0 / H, eps=1e-5), 16)
                row["wo_plain"] = G._time(lambda i: G._tgemm(ext, o, wo[i % copies], G.EPI_PLAIN, p, y=y[:, :H]), 16)
                rr = r.clone()
                row["wo_resadd"] = G._time(lambda i: G._tgemm(ext, o, wo[i % copies], G.EPI_RESADD, p, y=rr,
                                                              ssq_out=ssq), 16)
                row["gu_plain"] = G._time(lambda i: G._tgemm(ext, r, wgu[i % copies], G.EPI_PLAIN, p, y=y), 16)
                row["gu_swiglu"] = G._time(lambda i: G._tgemm(ext, r, wgu[i % copies], G.EPI_SWIGLU, p, y=act,
                                                              ssq_in=ssq, ssq_n=8, norm_scale=1.0 / H, eps=1e-5), 16)
            except Exception as e:  # noqa: BLE001
                row["error"] = str(e)[:100]
            print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in row.items()}), flush=True)


if __name__ == "__main__":
    main()
