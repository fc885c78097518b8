"""Host-only simulation of the flagship's KV block traffic through the native block manager
(csrc/runtime/block_manager.h), to measure where new blocks land (run continuation, a wholly free
segment, or scattered) without a GPU.

Workload (as bench.py's event driver): P concurrent growing conversations; each turn re-sends the
whole history (the reference's protocol, src/router.py:161-167 -> src/devices/nano_api.py:49-52),
so the prefix cache matches the previous turn's prompt blocks; the answer's tokens usually do NOT
re-tokenize to the generated ids (random-init models emit arbitrary ids), so the previous turn's
decode blocks go stale in the LRU.  Continuous batching: one token per active sequence per step; a
finished turn frees its sequence and starts the next at once.  The pool is sized so the cached
history fills it (LRU eviction active), as on the GPU.
Usage: python scripts/kv_placement_sim.py [--convs 128] [--steps 6000]
"""
import argparse
import os
import sys
import json
import random

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_llm_amd.engine import _runtime


def simulate(convs=96, steps=5000, pool_blocks=None, seed=0, retok_same=0.3, contiguous=True, bs=16, ctx_cap=7000,
             gap=(0, 0)):
    rng = random.Random(seed)
    pool = pool_blocks or convs * 360
    bm = _runtime.BlockManager(pool, bs, True, int(contiguous) if not isinstance(contiguous, bool) else (2 if contiguous else 0))
    hist = [[rng.randrange(32000) for _ in range(rng.randrange(20, 80))] for _ in range(convs)]
    active = {}
    waiting = {}                 # conversation -> step at which its next turn is dispatched
    nid = 0
    step = 0

    def start(c):
        nonlocal nid
        prompt = hist[c] + [rng.randrange(32000) for _ in range(rng.randrange(10, 40))]
        if len(prompt) > ctx_cap:           # conversation reset (bounded context)
            prompt = prompt[-rng.randrange(40, 120):]
        table, _ = bm.allocate(nid, prompt)
        if not table:
            return False
        bm.commit(nid, len(prompt))
        active[c] = {"id": nid, "prompt": prompt, "gen": [], "left": rng.randrange(16, 300)}
        nid += 1
        return True

    for c in range(convs):
        start(c)
    st0 = bm.stats()
    for step in range(steps):
        cs = list(active)
        toks = [rng.randrange(32000) for _ in cs]
        slots = bm.commit_append([active[c]["id"] for c in cs], toks, [1] * len(cs))
        for c, tok, slot in zip(cs, toks, slots):
            a = active[c]
            if slot < 0:
                a["left"] = 0
            else:
                a["gen"].append(tok)
                a["left"] -= 1
            if a["left"] <= 0:
                bm.free(a["id"])
                gen = a["gen"] if rng.random() < retok_same else [rng.randrange(32000) for _ in a["gen"]]
                hist[c] = a["prompt"] + gen
                del active[c]
                # the driver dispatches the next turn after a routing / admission gap, during which
                # the conversation's blocks sit in the LRU (the bench: admission every 16 steps)
                waiting[c] = step + rng.randint(*gap)
        for c in range(convs):             # dispatch due turns; re-admit any that could not allocate
            if c not in active and waiting.get(c, -1) <= step:
                if start(c):
                    waiting.pop(c, None)
    st1 = bm.stats()
    d = {k: st1.get(k, 0) - st0.get(k, 0) for k in ("contiguous_allocs", "segment_allocs", "fresh_allocs",
                                                    "prefix_hit_tokens", "prompt_tokens", "inplace_evictions",
                                                    "roomy_segment_allocs", "run_miss_first", "run_miss_held",
                                                    "run_miss_hot")}
    err = bm.check_invariants()
    return {"pool_blocks": pool, "convs": convs, "new_blocks": d["fresh_allocs"],
            "run_share": round(d["contiguous_allocs"] / max(1, d["fresh_allocs"]), 3),
            "segment_share": round(d["segment_allocs"] / max(1, d["fresh_allocs"]), 3),
            "roomy_segment_share": round(d["roomy_segment_allocs"] / max(1, d["fresh_allocs"]), 3),
            "inplace_share": round(d["inplace_evictions"] / max(1, d["fresh_allocs"]), 3),
            "miss_first_share": round(d["run_miss_first"] / max(1, d["fresh_allocs"]), 3),
            "miss_held_share": round(d["run_miss_held"] / max(1, d["fresh_allocs"]), 3),
            "miss_hot_share": round(d["run_miss_hot"] / max(1, d["fresh_allocs"]), 3),
            "prefix_hit_rate": round(d["prefix_hit_tokens"] / max(1, d["prompt_tokens"]), 3),
            "invariants": err or "ok"}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--convs", type=int, default=96)
    ap.add_argument("--steps", type=int, default=5000)
    ap.add_argument("--pool", type=int, default=0)
    ap.add_argument("--gap", type=int, nargs=2, default=(5, 40), help="turn gap range in steps")
    a = ap.parse_args()
    for gap in ((0, 0), tuple(a.gap)):
        for mode in (0, 1, 2):   # block_manager.h placement: 0 LIFO, 1 round-5 runs, 2 round-6 (default)
            print(json.dumps(dict(simulate(a.convs, a.steps, a.pool or None, contiguous=mode, gap=gap),
                                  placement=mode, gap=list(gap))), flush=True)
