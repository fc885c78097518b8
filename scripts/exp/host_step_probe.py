"""Single-stream decode: wall ms per token vs the GPU step time, and where the host time goes.

Runs LLMEngine.generate on ONE prompt (ignore_eos, N new tokens) in the calling thread, prints
wall ms/token for greedy and sampled decoding, the engine timers, and a cProfile top list of the
sampled run (1x MI355X).  The GPU-only step time of the same bucket comes from
scripts/microbench.py --what decode.
"""
import cProfile
import io
import json
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from distributed_llm_amd.engine.llm_engine import LLMEngine  # noqa: E402
from distributed_llm_amd.engine.sampling import SamplingParams  # noqa: E402


def run(eng, sp, prompt):
    t0 = dict(eng.timers)
    torch.cuda.synchronize()
    t = time.perf_counter()
    out = eng.generate([prompt], sp)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    tim = {k: round(eng.timers[k] - t0.get(k, 0.0), 4) for k in eng.timers}
    return dt, out[0], tim


def main():
    n = int(os.environ.get("PROBE_TOKENS", "256"))
    eng = LLMEngine(os.environ.get("PROBE_MODEL", "tinyllama-1.1b"), device="cuda", kv_cache_gb=4.0, max_num_seqs=8)
    eng.capture_all(max_bs=8)
    prompt = list(range(100, 100 + int(os.environ.get("PROBE_PROMPT", "512"))))
    for name, sp in (("greedy", SamplingParams(max_new_tokens=n, ignore_eos=True)),
                     ("sampled", SamplingParams(max_new_tokens=n, temperature=0.8, top_k=40, top_p=0.9,
                                                ignore_eos=True))):
        run(eng, sp, prompt)   # warm
        dt, o, tim = run(eng, sp, prompt)
        print(json.dumps({"mode": name, "pipeline": eng._pipeline_ok(), "tokens": o.num_generated,
                          "ms_per_token": round(dt * 1000 / o.num_generated, 3), "timers_s": tim}), flush=True)
    pr = cProfile.Profile()
    pr.enable()
    run(eng, SamplingParams(max_new_tokens=n, temperature=0.8, top_k=40, top_p=0.9, ignore_eos=True), prompt)
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    print(s.getvalue())


if __name__ == "__main__":
    main()
