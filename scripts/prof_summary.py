"""Summarise a rocprofv3 --stats kernel_stats.csv into a compact markdown table."""
import csv
import sys

path = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time: {tot/1e6:.1f} ms over {sum(int(r['Calls']) for r in rows)} dispatches\n")
print("| % | total ms | calls | avg us | kernel |")
print("|---|---|---|---|---|")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    name = r["Name"]
    name = name if len(name) < 110 else name[:107] + "..."
    print(f"| {float(r['Percentage']):.1f} | {float(r['TotalDurationNs'])/1e6:.2f} | {r['Calls']} | "
          f"{float(r['AverageNs'])/1e3:.1f} | `{name}` |")
