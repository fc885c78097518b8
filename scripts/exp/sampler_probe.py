"""Batch-1 sampler cost vs the logit distribution (round 4).  One graph of 20 back-to-back sampler
launches per case; us per launch for the one-workgroup-per-row kernel and the split-vocab kernel.
Also reports, for the decode microbench's own random-init TinyLlama, the logits' spread."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from distributed_llm_amd import ops  # noqa: E402

DEV = "cuda"
ext = ops._native(torch.empty(1, device=DEV))


def timed(fn, reps=20, iters=10):
    s = torch.cuda.Stream()
    fn()
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / (reps * iters)


def case(name, lg, temp, k):
    B, V = lg.shape
    T = torch.full((B,), temp, device=DEV)
    P_ = torch.full((B,), 0.9, device=DEV)
    K = torch.full((B,), k, dtype=torch.int32, device=DEV)
    S = torch.tensor([3], dtype=torch.int32, device=DEV)
    o = torch.empty(B, dtype=torch.int32, device=DEV)
    one = timed(lambda: ext.sample_rows(lg, T, P_, K, S, o))
    split = timed(lambda: ops.sample_rows(lg, T, P_, K, S, out=o))
    print(json.dumps({"case": name, "B": B, "V": V, "temp": temp, "k": k, "one_wg_us": round(one, 2),
                      "split_us": round(split, 2)}), flush=True)


def main():
    torch.manual_seed(0)
    for V in (32000, 128256):
        g = torch.randn(1, V, device=DEV)
        for sd in (1.0, 0.05):
            case(f"gauss{sd}", (g * sd).to(torch.bfloat16), 0.8, 40)
        case("gauss1_greedy", g.to(torch.bfloat16), 0.0, 40)
        case("gauss1_k256", g.to(torch.bfloat16), 0.8, 0)
        case("ints0-3", torch.randint(0, 4, (1, V), device=DEV).to(torch.bfloat16), 0.8, 40)
    # the random-init TinyLlama's own logits for one decode position
    from distributed_llm_amd.engine.llm_engine import LLMEngine
    eng = LLMEngine("tinyllama-1.1b", device=DEV, kv_cache_gb=2.0, max_num_seqs=8, max_model_len=2048)
    m = eng.model
    h = torch.randn(1, m.cfg.hidden, device=DEV).to(torch.bfloat16) if hasattr(m, "cfg") else None
    lg = m.logits(h) if h is not None else None
    if lg is not None:
        lf = lg.float()
        top = torch.topk(lf[0], 64).values
        print(json.dumps({"model_logits": {"std": round(float(lf.std()), 4), "max": round(float(lf.max()), 4),
                                           "top1_top40_top64": [round(float(top[0]), 4), round(float(top[39]), 4),
                                                                round(float(top[63]), 4)],
                                           "distinct_top64": int(torch.unique(top).numel())}}), flush=True)
        case("tinyllama_random_init", lg.contiguous(), 0.8, 40)


if __name__ == "__main__":
    main()
