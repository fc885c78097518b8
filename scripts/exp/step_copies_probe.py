"""What the per-step host<->device copies around a batch-1 decode graph cost (1x MI355X).

Replays the engine's bucket-1 decode graph 200 times in a pipelined loop (step k+1 enqueued before
waiting on step k, as LLMEngine._decode_burst does) with different subsets of the per-step copies:
  meta  : H2D of the step metadata (pinned -> dec_dev)
  items : H2D of the attention work list
  ids   : D2D gather of the previous step's sampled tokens into the input ids
  out   : D2H of the sampled tokens into pinned memory + event (the host needs them)
and prints ms per step for each variant.
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from distributed_llm_amd.engine.llm_engine import LLMEngine  # noqa: E402
from distributed_llm_amd.engine.sampling import SamplingParams  # noqa: E402


def main():
    eng = LLMEngine("tinyllama-1.1b", device="cuda", kv_cache_gb=4.0, max_num_seqs=8)
    eng.capture_all(max_bs=8)
    # one real decode so the metadata buffers hold a valid batch-1 step
    eng.generate([list(range(100, 612))], SamplingParams(max_new_tokens=4, ignore_eos=True))
    g = eng._graphs[1]
    meta_n = 4096
    pin = eng._dec_bufs[0][0]
    items_pin = eng._items_bufs[0][0]
    outs = [torch.zeros(8, dtype=torch.int32, pin_memory=True) for _ in range(2)]
    evs = [torch.cuda.Event(), torch.cuda.Event()]
    n = 200
    for name, flags in (("graph only", ()), ("meta", ("meta",)), ("items", ("items",)), ("ids", ("ids",)),
                        ("out", ("out",)), ("meta+items+ids+out (engine)", ("meta", "items", "ids", "out")),
                        ("meta+out", ("meta", "out"))):
        torch.cuda.synchronize()
        t = time.perf_counter()
        prev = None
        for i in range(n):
            if "meta" in flags:
                eng.dec_dev[:meta_n].copy_(pin[:meta_n], non_blocking=True)
            if "items" in flags:
                eng.items_dev[:64].copy_(items_pin[:64], non_blocking=True)
            if "ids" in flags:
                eng.d_ids[:1].copy_(eng.d_out[:1])
            g.replay()
            if "out" in flags:
                outs[i & 1][:1].copy_(eng.d_out[:1], non_blocking=True)
                evs[i & 1].record()
                if prev is not None:
                    prev.synchronize()
                prev = evs[i & 1]
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) * 1000 / n
        print(json.dumps({"variant": name, "ms_per_step": round(ms, 4)}), flush=True)


if __name__ == "__main__":
    main()
