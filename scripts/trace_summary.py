"""Summarise a Chrome trace written by distributed_llm_amd.utils.tracing (bench.py --trace PATH).

Prints a markdown table per span name: count, total / mean / max ms, host vs GPU lanes, and the
share of the decode-step host span that the GPU spent executing the decode graph.
Usage: python scripts/trace_summary.py trace.json [title]
"""
import json
import sys


def main() -> None:
    path = sys.argv[1]
    title = sys.argv[2] if len(sys.argv) > 2 else path
    evs = json.load(open(path))["traceEvents"]
    agg = {}
    for e in evs:
        if e.get("ph") != "X":
            continue
        lane = "gpu" if str(e.get("tid", "")).startswith("gpu:") else "host"
        a = agg.setdefault((e["name"], lane), [0, 0.0, 0.0])
        d = e["dur"] / 1000.0
        a[0] += 1
        a[1] += d
        a[2] = max(a[2], d)
    print(f"# trace summary: {title}\n")
    print("| span | lane | count | total ms | mean ms | max ms |")
    print("|---|---|---|---|---|---|")
    for (name, lane), (n, tot, mx) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"| {name} | {lane} | {n} | {tot:.1f} | {tot / n:.3f} | {mx:.2f} |")
    step = agg.get(("engine.decode", "host"))
    gpu = agg.get(("engine.decode_forward", "gpu"))
    if step and gpu:
        print(f"\nGPU busy share of decode steps (decode graph time / decode step wall time): "
              f"{gpu[1] / step[1]:.3f}")
    cs = [e for e in evs if e.get("ph") == "C" and e["name"] == "engine.batch"]
    if cs:
        run = [c["args"]["running"] for c in cs]
        print(f"decode batch: mean {sum(run) / len(run):.1f}, max {max(run)} over {len(run)} steps")


if __name__ == "__main__":
    main()
