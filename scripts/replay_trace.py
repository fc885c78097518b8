"""One decode-graph replay from a rocprofv3 kernel trace: per-kernel time and launch gaps.

Usage: python scripts/replay_trace.py <kernel_trace.csv> [first_kernel_substring]

Takes the dispatches between the last two occurrences of the step's first kernel (default
``embed_kernel``: every decode graph starts with the token-embedding gather), then prints a
per-kernel-name table (calls, total us, avg us) and the step's busy vs wall time, so launch gaps
inside a captured step show up as wall - busy.
"""
import csv
import sys
from collections import OrderedDict


def main() -> None:
    path = sys.argv[1]
    first = sys.argv[2] if len(sys.argv) > 2 else "embed_kernel"
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
    if len(idx) < 2:
        sys.exit(f"fewer than two '{first}' dispatches in {path}")
    step = rows[idx[-2]:idx[-1]]
    t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step)
    agg = OrderedDict()
    for r in step:
        name = r["Kernel_Name"]
        name = name if len(name) < 100 else name[:97] + "..."
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        c, s = agg.get(name, (0, 0.0))
        agg[name] = (c + 1, s + d)
    print(f"one replay: {len(step)} dispatches, wall {(t1 - t0) / 1e3:.1f} us, kernels busy {busy / 1e3:.1f} us, "
          f"gaps {(t1 - t0 - busy) / 1e3:.1f} us ({(t1 - t0 - busy) / 1e3 / max(1, len(step) - 1):.2f} us per launch)\n")
    print("| calls | total us | avg us | kernel |")
    print("|---|---|---|---|")
    for name, (c, s) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"| {c} | {s:.1f} | {s / c:.2f} | `{name}` |")


if __name__ == "__main__":
    main()
