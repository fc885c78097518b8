"""What do a pipelined decode step's host copies cost on the GPU timeline?  (round 4)

The flagship's gap analysis (profiles/r4_driver_window_gaps.md) charges ~300 us of GPU idle per
decode step to the copies around the graph: the D2H read-out of the sampled tokens and the H2D
staging of the next step's inputs.  Decode graph of B rows at context C (TinyLlama), per step:
  replay     : the graph alone
  +readout   : graph, then d_out -> pinned host (non_blocking), as _read_out does
  +stage     : graph, read-out, then pinned -> device input copies (dec + items), as _prep_decode does
  ingraph    : the same copies captured INSIDE the graph (memcpy nodes), alternating two pinned
               buffers like the engine's parity
ms per step over a back-to-back loop, host never waiting except at the end.
"""
import json
import os
import sys

import torch

ROOT = os.path.join(os.path.dirname(__file__), "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts", "exp"))
from distributed_llm_amd.engine.llm_engine import LLMEngine  # noqa: E402
from two_graph_overlap import prepare, timed  # noqa: E402


def main():
    B = int(os.environ.get("PROBE_B", "496"))
    C = int(os.environ.get("PROBE_C", "1800"))
    eng = LLMEngine("tinyllama-1.1b", device="cuda", kv_cache_gb=float(os.environ.get("PROBE_KV_GB", "40")),
                    max_num_seqs=B)
    g = prepare(eng, B, C, 10_000_000)
    bs = eng._bucket(B)
    n_dec = eng.dec_dev.numel()
    n_items = eng.items_dev.numel() if getattr(eng, "items_dev", None) is not None else 0
    pin_in = [torch.empty(n_dec, dtype=eng.dec_dev.dtype, pin_memory=True) for _ in range(2)]
    pin_out = [torch.empty(bs + 1, dtype=eng.d_out.dtype, pin_memory=True) for _ in range(2)]
    pin_it = [torch.empty(max(n_items, 1), dtype=eng.items_dev.dtype, pin_memory=True) for _ in range(2)] \
        if n_items else None
    for p in range(2):
        pin_in[p].copy_(eng.dec_dev.cpu())
        if pin_it:
            pin_it[p].copy_(eng.items_dev.cpu())
    state = {"p": 0}
    K = 10

    def loop(fn):
        def run():
            for _ in range(K):
                fn()
        return run

    def replay():
        g.replay()

    def readout():
        g.replay()
        pin_out[state["p"]].copy_(eng.d_out[:bs + 1], non_blocking=True)
        state["p"] ^= 1

    def stage():
        p = state["p"]
        eng.dec_dev.copy_(pin_in[p], non_blocking=True)
        if pin_it:
            eng.items_dev.copy_(pin_it[p], non_blocking=True)
        g.replay()
        pin_out[p].copy_(eng.d_out[:bs + 1], non_blocking=True)
        state["p"] ^= 1

    # the same copies inside one graph per parity: H2D nodes, the decode step's body, D2H node
    graphs = []
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    for p in range(2):
        gp = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gp, pool=eng._graph_pool, stream=s):
            eng.dec_dev.copy_(pin_in[p], non_blocking=True)
            if pin_it:
                eng.items_dev.copy_(pin_it[p], non_blocking=True)
            eng._decode_forward(bs)
            pin_out[p].copy_(eng.d_out[:bs + 1], non_blocking=True)
        graphs.append(gp)
    torch.cuda.current_stream().wait_stream(s)

    def ingraph():
        graphs[state["p"]].replay()
        state["p"] ^= 1

    res = {"B": B, "C": C, "bucket": bs, "dec_words": n_dec, "item_words": n_items, "steps_per_trial": K}
    for name, fn in (("replay", replay), ("readout", readout), ("stage", stage), ("ingraph", ingraph),
                     ("replay_2", replay), ("stage_2", stage), ("ingraph_2", ingraph)):
        res[name + "_ms_per_step"] = round(timed(loop(fn), 5) / K, 4)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
