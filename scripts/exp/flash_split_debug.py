"""Where do non-finite outputs of the split-KV flash prefill land?  (debug, round 4)"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
from distributed_llm_amd import ops  # noqa: E402
from distributed_llm_amd.ops import reference as ref  # noqa: E402
from test_flash_gpu import _case  # noqa: E402

for sp in ("1", "2", "4"):
    os.environ["DLLM_FLASH_SPLITS"] = sp
    for nan in (True, False):
        d, nq, nkv = 64, 32, 4
        seqs = [(300, 300), (37, 37), (200, 777), (129, 129), (1, 50), (16, 33)]
        q, kc, vc, bt, qs, ql, cx = _case(d, nq, nkv, seqs, seed=d + nq)
        if not nan:
            kc, vc = kc.nan_to_num(0.0), vc.nan_to_num(0.0)
        ts, tt = ops.flash_tiles(ql.tolist(), nq // nkv)
        C = lambda t: t.cuda()
        got = ops.flash_attention(C(q), C(kc), C(vc), C(bt), C(qs), C(ql), C(cx), C(torch.tensor(ts, dtype=torch.int32)),
                                  C(torch.tensor(tt, dtype=torch.int32)), causal=True).cpu().float()
        want = ref.paged_attention(q, kc.nan_to_num(0.0), vc.nan_to_num(0.0), bt, qs, ql, cx, 1.0 / math.sqrt(d), True).float()
        bad = ~torch.isfinite(got)
        tok = bad.any(-1).any(-1).nonzero().flatten().tolist()
        err = (got.nan_to_num(99) - want).abs().amax(-1).amax(-1)
        print(f"splits={sp} nan_tails={nan}: nonfinite tokens {len(tok)} first {tok[:12]}; "
              f"max err finite {float(err[~bad.any(-1).any(-1)].max()):.4f}; worst tokens {err.topk(5).indices.tolist()}",
              flush=True)
