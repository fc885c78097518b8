"""Attribute __amd_rocclr_copyBuffer dispatches in a rocprofv3 kernel trace: count / time by queue
and thread, grid size, and the kernel that ran before each copy on the same queue.
Usage: python scripts/exp/copy_attrib.py <kernel_trace.csv>"""
import collections
import csv
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    last = {}
    by = collections.defaultdict(lambda: [0, 0.0])
    prev = collections.Counter()
    grids = collections.Counter()
    threads = collections.Counter()
    for r in rows:
        q = r.get("Queue_Id", "?")
        name = r["Kernel_Name"]
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if "copyBuffer" in name:
            key = (q, r.get("Thread_Id", "?"))
            by[key][0] += 1
            by[key][1] += dur
            prev[(q, last.get(q, "<none>")[:70])] += 1
            grids[(q, r.get("Grid_Size", r.get("Grid_Size_X", "?")))] += 1
        last[q] = name
    print("copyBuffer by (queue, thread): count, total us")
    for k, (n, t) in sorted(by.items(), key=lambda kv: -kv[1][1]):
        print(f"  {k}: {n}, {t:.0f} us, avg {t / n:.1f}")
    print("grid sizes (queue, grid): count")
    for k, n in grids.most_common(12):
        print(f"  {k}: {n}")
    print("previous kernel on the same queue: count")
    for k, n in prev.most_common(15):
        print(f"  {k}: {n}")
    qs = collections.Counter(r.get("Queue_Id", "?") for r in rows)
    print("dispatches per queue:", dict(qs))


if __name__ == "__main__":
    main(sys.argv[1])
