"""GPU idle time between kernels from a rocprofv3 kernel-trace CSV.

Usage: python scripts/gap_summary.py <kernel_trace.csv> [skip_fraction]

Busy time is the union of kernel intervals; every gap between consecutive intervals (the GPU ran
nothing) is charged to the pair (kernel before -> kernel after), so host-side stalls show up by
where they happen in the step (e.g. before a graph's first kernel, around prefill, after the
sampler).  ``skip_fraction`` drops the first part of the run (start-up, tuning, capture)."""
import csv
import sys
from collections import defaultdict


def short(name: str) -> str:
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:70]


def main():
    # argv[1]: kernel-trace CSV, or several joined by commas (e.g. + the memory-copy trace: its
    # rows are named by their direction, so SDMA copies show up between the kernels)
    paths = sys.argv[1].split(",")
    skip = float(sys.argv[2]) if len(sys.argv) > 2 else 0.3
    rows = []
    for path in paths:
      with open(path) as f:
        for r in csv.DictReader(f):
            k = r.get("Kernel_Name") or r.get("KernelName") or r.get("Name")
            if not k and (r.get("Direction") or r.get("Kind")):
                k = "COPY " + (r.get("Direction") or r.get("Kind"))
            s = r.get("Start_Timestamp") or r.get("BeginNs") or r.get("Start")
            e = r.get("End_Timestamp") or r.get("EndNs") or r.get("End")
            q = r.get("Stream_Id") or r.get("Queue_Id") or ""
            if k and s and e:
                rows.append((int(s), int(e), short(k) + (f" [q{q}]" if q else "")))
    rows.sort()
    t0, t1 = rows[0][0], max(e for _, e, _ in rows)
    # skip <= 1: fraction of the run to drop; skip > 1: keep only the last `skip` seconds
    cut = t0 + skip * (t1 - t0) if skip <= 1 else t1 - int(skip * 1e9)
    rows = [r for r in rows if r[0] >= cut]
    busy, gaps = 0, defaultdict(lambda: [0, 0])
    cur_s, cur_e, cur_k = rows[0]
    hist = defaultdict(int)
    for s, e, k in rows[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            g = s - cur_e
            gaps[(cur_k, k)][0] += g
            gaps[(cur_k, k)][1] += 1
            b = "<2us" if g < 2000 else "2-5us" if g < 5000 else "5-20us" if g < 20000 else "20-100us" if g < 100000 else ">=100us"
            hist[b] += g
            cur_s, cur_e, cur_k = s, e, k
        else:
            cur_e, cur_k = max(cur_e, e), k if e >= cur_e else cur_k
    busy += cur_e - cur_s
    span = cur_e - rows[0][0]
    idle = span - busy
    what = f"first {skip:.0%} of the run skipped" if skip <= 1 else f"last {skip:g} s of the run"
    print(f"window {span / 1e9:.3f} s ({what}): GPU busy {busy / 1e9:.3f} s "
          f"({100 * busy / span:.1f} %), idle {idle / 1e9:.3f} s\n")
    print("| gap size | idle s | share of idle |\n|---|---|---|")
    for b in ("<2us", "2-5us", "5-20us", "20-100us", ">=100us"):
        print(f"| {b} | {hist[b] / 1e9:.3f} | {100 * hist[b] / max(idle, 1):.1f} % |")
    per = defaultdict(lambda: [0, 0])
    for s_, e_, k in rows:
        per[k][0] += e_ - s_
        per[k][1] += 1
    tot = sum(v[0] for v in per.values())
    print("\n| kernel | ms in window | calls | avg us | share of kernel time |\n|---|---|---|---|---|")
    for k, (t, n) in sorted(per.items(), key=lambda x: -x[1][0])[:15]:
        print(f"| `{k}` | {t / 1e6:.1f} | {n} | {t / n / 1e3:.1f} | {100 * t / max(tot, 1):.1f} % |")
    print("\n| idle ms | gaps | mean us | kernel before | kernel after |\n|---|---|---|---|---|")
    for (a, b), (g, n) in sorted(gaps.items(), key=lambda x: -x[1][0])[:25]:
        print(f"| {g / 1e6:.1f} | {n} | {g / n / 1e3:.1f} | `{a}` | `{b}` |")
    # the neighbourhood of the first mid-size (100-400 us) idle gap in the second half of the window
    prev_e = rows[0][1]
    for i in range(len(rows) // 2, len(rows)):
        g = rows[i][0] - max(e for _, e, _ in rows[max(0, i - 8):i]) if i > 0 else 0
        if 100_000 <= g <= 400_000:
            print(f"\nAround a {g / 1e3:.0f} us gap (us relative to the row after it):\n")
            print("| t | dur | kernel |\n|---|---|---|")
            for s_, e_, k in rows[max(0, i - 25):i + 12]:
                print(f"| {(s_ - rows[i][0]) / 1e3:.1f} | {(e_ - s_) / 1e3:.1f} | `{k}` |")
            break
    # a timeline excerpt from the middle of the window: what runs between two idle gaps
    mid = len(rows) // 2
    print("\nTimeline excerpt (us from the first row; gap = idle before the row):\n")
    print("| t | dur | gap | kernel |\n|---|---|---|---|")
    base, prev_e = rows[mid][0], rows[mid][0]
    for s_, e_, k in rows[mid:mid + 160]:
        print(f"| {(s_ - base) / 1e3:.1f} | {(e_ - s_) / 1e3:.1f} | {max(0, s_ - prev_e) / 1e3:.1f} | `{k}` |")
        prev_e = max(prev_e, e_)


if __name__ == "__main__":
    main()
