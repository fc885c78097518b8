"""Is there GPU idle time BETWEEN back-to-back decode graph replays?  (round 5)

The driver-window trace (profiles/r5_driver_window_gaps.md) shows a ~170 us gap between one decode
step's last kernel (step_store) and the next step's first (step_fetch) on most steps, although the
step loop has the next step queued ~5 ms ahead (DLLM_DIAG=sync: wait p50 4.97 ms).  This replays
the engine's real decode graph (TinyLlama, B rows at context C) K times with nothing else on the
device: A = back to back, B = with an event recorded after each replay (as _read_out does),
C = alternating the two staging-buffer parities (as the pipelined burst does).  ms per step; under
rocprofv3 --kernel-trace the per-step kernel sum and the gaps come from scripts/gap_summary.py."""
import json
import os
import sys
import time

import torch

ROOT = os.path.join(os.path.dirname(__file__), "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts", "exp"))
from distributed_llm_amd.engine.llm_engine import LLMEngine  # noqa: E402
from two_graph_overlap import prepare  # noqa: E402


def main():
    B = int(os.environ.get("PROBE_B", "496"))
    C = int(os.environ.get("PROBE_C", "1800"))
    K = int(os.environ.get("PROBE_K", "40"))
    eng = LLMEngine("tinyllama-1.1b", device="cuda", kv_cache_gb=40.0, max_num_seqs=B)
    g0 = prepare(eng, B, C, 10_000_000)
    bs = eng._bucket(B)
    # parity 1: same staging contents (graph I/O reads the pinned buffer of its parity)
    for a, b in zip(eng._dec_bufs[1], eng._dec_bufs[0]):
        if hasattr(a, "copy_"):
            a.copy_(b)
        else:
            a[:] = b
    if getattr(eng, "_items_bufs", None):
        eng._items_bufs[1][0].copy_(eng._items_bufs[0][0])
    g1 = eng._graphs.get(eng._gkey(bs, 1)) or eng._capture(bs, 1)
    ev = [torch.cuda.Event(), torch.cuda.Event()]

    def run(mode):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for i in range(K):
            g = g1 if (mode == "C" and i % 2) else g0
            g.replay()
            if mode in ("B", "C"):
                ev[i % 2].record()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) * 1000 / K

    for m in ("A", "B", "C"):
        run(m)
    res = {m: round(min(run(m) for _ in range(3)), 3) for m in ("A", "B", "C")}
    print(json.dumps({"B": B, "C": C, "K": K, "ms_per_step": res}), flush=True)


if __name__ == "__main__":
    main()
