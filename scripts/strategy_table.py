"""Per-strategy table (BASELINE metric: routed p50 latency + tokens/s per strategy) from
gpurun_out/strat/<strategy>.log, written by scripts/strategy_sweep.sh."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
d = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "strat")
print("| strategy | routed tok/s | vs best published 10.57 tok/s | p50 turn (ms) | p90 (ms) | small-tier share | "
      "avg decode batch | mean routing overhead (ms) | J / token |")
print("|---|---|---|---|---|---|---|---|---|")
for s in ["token", "heuristic", "semantic", "perf", "hybrid"]:
    f = os.path.join(d, f"{s}.log")
    if not os.path.exists(f):
        continue
    lines = [l for l in open(f) if l.startswith('{"metric"')]
    if not lines:
        continue
    r = json.loads(lines[-1])
    print(f"| {s} | {r['value']:,.0f} | x{r['vs_baseline']:,.0f} | {r['p50_latency_ms']:,.0f} | {r['p90_latency_ms']:,.0f} | "
          f"{r['small_tier_share']} | {r['avg_decode_batch']} | {r['routing_overhead_ms_mean']} | {r.get('j_per_token', '-')} |")
