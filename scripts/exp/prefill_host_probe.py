"""Host cost of launching one admission prefill chunk (round 4).

With in-burst joins the GPU idles when the step loop's host work at an admission outlasts the
decode steps already queued (profiles/r4_driver_window_gaps.md: t_prefill ~7.8 ms of host per
admission).  This times the host side of one chunk -- the flagship's shape: P sequences x Q new
tokens behind X cached -- through the engine's own `_prefill_launch` (metadata, staging, the eager
layer loop, the first-token sampler), then prints a cProfile of it."""
import cProfile
import io
import json
import os
import pstats
import sys
import time

import torch

ROOT = os.path.join(os.path.dirname(__file__), "..", "..")
sys.path.insert(0, ROOT)
from distributed_llm_amd.engine.llm_engine import LLMEngine, _Seq  # noqa: E402
from distributed_llm_amd.engine.sampling import SamplingParams  # noqa: E402


def make_chunk(eng, P, Q, X, base):
    seqs = []
    for i in range(P):
        s = _Seq(id=base + i, prompt=[5 + (i * 7 + j) % 1000 for j in range(X + Q)],
                 params=SamplingParams(max_new_tokens=8, temperature=0.8, top_k=40, top_p=0.9),
                 arrival=time.perf_counter())
        seqs.append(s)
    waiting, pre = list(seqs), []
    eng._admit(waiting, pre, 0)
    for s in pre:                    # as if the first X tokens were a prefix-cache hit
        s.num_computed = max(s.num_computed, X)
    return pre


def main():
    P, Q, X = (int(os.environ.get(k, d)) for k, d in (("PROBE_P", "30"), ("PROBE_Q", "130"), ("PROBE_X", "1700")))
    eng = LLMEngine("tinyllama-1.1b", device="cuda", kv_cache_gb=16.0, max_num_seqs=64)
    res = {"seqs": P, "new_tokens": P * Q, "cached": X}
    times = []
    prof = cProfile.Profile()
    for it in range(6):
        pre = make_chunk(eng, P, Q, X, 1_000_000 * (it + 1))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if it == 5:
            prof.enable()
        h = eng._prefill_launch(pre)
        if it == 5:
            prof.disable()
        t1 = time.perf_counter()
        eng._prefill_finish(h)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        times.append((round((t1 - t0) * 1e3, 3), round((t2 - t0) * 1e3, 3)))
        for s in pre:
            eng._release(s)
    res["host_launch_ms_and_total_ms"] = times
    print(json.dumps(res), flush=True)
    out = io.StringIO()
    pstats.Stats(prof, stream=out).sort_stats("cumulative").print_stats(30)
    print(out.getvalue())


if __name__ == "__main__":
    main()
