"""Per-step kernel breakdown of a replayed decode graph from a rocprofv3 kernel-trace DB:
finds the period of the trailing dispatch sequence (one graph replay), then averages each kernel's
duration and the step's wall time / idle share over the last R replays.
Usage: python scripts/exp/step_kernels.py gpurun_out/r6k/b4/p_results.db [R]"""
import sqlite3
import sys
from collections import defaultdict


def main(db, reps=10):
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    names = [r[0] for r in rows]
    n = len(names)
    period = None
    for p in range(8, 2000):
        if n >= 3 * p and names[n - p:] == names[n - 2 * p:n - p] == names[n - 3 * p:n - 2 * p]:
            period = p
            break
    if period is None:
        raise SystemExit("no period found")
    tail = rows[n - reps * period:]
    per = defaultdict(float)
    cnt = defaultdict(int)
    for name, s, e in tail:
        short = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:90]
        per[short] += (e - s) / reps / 1000.0
        cnt[short] += 1
    wall = (tail[-1][2] - tail[0][1]) / reps / 1000.0
    busy = sum(per.values())
    print(f"period {period} dispatches per step; wall {wall:.1f} us, kernel sum {busy:.1f} us "
          f"({100 * busy / wall:.1f} % busy)")
    for k, v in sorted(per.items(), key=lambda kv: -kv[1]):
        print(f"{v:8.1f} us  {cnt[k] // reps:4d}x  {k}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 10)
