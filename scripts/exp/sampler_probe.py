"""Fused sampler (sample_rows_kernel) time per launch at batch 1-512, V = 32000 (1x MI355X).

Random-normal bf16 logits (std 3), temperature 0.8, top-k 40, top-p 0.9 (the large tier's
sampling); a hipGraph of 20 launches, us per launch.  Prints one JSON line per batch size.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from distributed_llm_amd import ops  # noqa: E402


def main():
    V = int(os.environ.get("PROBE_V", "32000"))
    for B in (1, 8, 64, 512):
        logits = (torch.randn(B, V, device="cuda") * 3).to(torch.bfloat16)
        for mode, t, k in (("sampled", 0.8, 40), ("greedy", 0.0, 0)):
            temp = torch.full((B,), t, device="cuda")
            tp = torch.full((B,), 0.9, device="cuda")
            tk = torch.full((B,), k, dtype=torch.int32, device="cuda")
            seed = torch.tensor([7], dtype=torch.int32, device="cuda")
            out = torch.empty(B, dtype=torch.int32, device="cuda")
            ops.sample_rows(logits, temp, tp, tk, seed, out)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            st = torch.cuda.Stream()
            st.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(st), torch.cuda.graph(g, stream=st):
                for _ in range(20):
                    ops.sample_rows(logits, temp, tp, tk, seed, out)
            torch.cuda.current_stream().wait_stream(st)
            g.replay()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            g.replay()
            e.record()
            torch.cuda.synchronize()
            print(json.dumps({"B": B, "V": V, "mode": mode, "us": round(s.elapsed_time(e) * 1000 / 20, 2)}), flush=True)


if __name__ == "__main__":
    main()
