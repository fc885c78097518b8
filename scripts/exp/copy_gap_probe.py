"""Does the per-step H2D metadata copy + D2H token copy + event around a decode graph replay leave
the GPU idle?  A small captured graph (a chain of elementwise kernels, ~1 ms of work) replayed
N times with the host always ahead, in four modes:
  graph       : replays only
  copies      : H2D (pinned, 8 KB) before and D2H (2 KB) + event record after every replay
  h2d_only / d2h_event : one side each
GPU time per iteration from events around the whole loop; idle per step = (t_mode - t_graph) / N."""
import json
import time

import torch


def main():
    dev = torch.device("cuda:0")
    x = torch.randn(1 << 22, device=dev)
    meta_h = torch.zeros(2048, dtype=torch.int32).pin_memory()
    meta_d = torch.zeros(2048, dtype=torch.int32, device=dev)
    out_h = torch.zeros(512, dtype=torch.int32).pin_memory()
    out_d = torch.zeros(512, dtype=torch.int32, device=dev)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        y = x * 1.0001
        with torch.cuda.graph(g, stream=s):
            for _ in range(40):
                y.mul_(1.0001).add_(0.5)
            out_d.copy_(meta_d[:512])
    torch.cuda.synchronize()
    N = 400
    res = {}
    for mode in ("graph", "copies", "h2d_only", "d2h_event", "graph"):
        evs = []
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        t0 = time.perf_counter()
        for i in range(N):
            if mode in ("copies", "h2d_only"):
                meta_d.copy_(meta_h, non_blocking=True)
            g.replay()
            if mode in ("copies", "d2h_event"):
                out_h.copy_(out_d, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
                evs.append(ev)
                if len(evs) > 2:
                    evs.pop(0).synchronize()   # like the pipelined burst: wait for step i-2
        e1.record()
        torch.cuda.synchronize()
        res[mode] = round(e0.elapsed_time(e1) * 1000.0 / N, 2)
        res[mode + "_host_us"] = round((time.perf_counter() - t0) * 1e6 / N, 2)
    res["idle_per_step_us_copies"] = round(res["copies"] - res["graph"], 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
