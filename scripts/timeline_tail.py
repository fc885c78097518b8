"""Tail of a rocprofv3 timeline (kernels + memory copies) with the idle gap before every op.

Usage: python scripts/timeline_tail.py <dir with *kernel_trace.csv [and *memory_copy_trace.csv]> [n_ops]

Prints the last ``n_ops`` GPU operations in start order (name, duration, idle gap since the previous
op ended) and a summary of where the GPU sat idle: the gaps before each op kind, so host-side or
copy-induced bubbles between hipGraph replays show up directly.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    ops = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY " + r.get("Direction", "")))
    ops.sort()
    return ops


def main():
    d = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    ops = load(d)[-n:]
    gaps = defaultdict(float)
    cnt = defaultdict(int)
    prev_end = ops[0][0]
    lines = []
    for s, e, name in ops:
        gap = max(0, s - prev_end) / 1e3
        key = name.split("(")[0].split("<")[0]
        gaps[key] += gap
        cnt[key] += 1
        lines.append(f"{(s - ops[0][0]) / 1e3:10.1f} us  dur {(e - s) / 1e3:7.2f}  gap {gap:7.2f}  {name}")
        prev_end = max(prev_end, e)
    wall = (ops[-1][1] - ops[0][0]) / 1e3
    busy = sum(e - s for s, e, _ in ops) / 1e3
    print(f"last {len(ops)} ops: wall {wall:.1f} us, busy {busy:.1f} us, idle {sum(gaps.values()):.1f} us\n")
    print("idle gap before each op kind (total us / count):")
    for k, v in sorted(gaps.items(), key=lambda kv: -kv[1])[:15]:
        print(f"  {v:9.1f}  {cnt[k]:5d}  {k}")
    print()
    print("\n".join(lines[-160:]))


if __name__ == "__main__":
    main()
