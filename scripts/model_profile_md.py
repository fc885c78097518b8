"""Render profiles/r2_<model>_bench_kernels.md from a scripts/gpu_model_bench.sh run
(gpurun_out/model_<model>/{bench.log, summary.md})."""
import json
import sys

m = sys.argv[1]
d = f"gpurun_out/model_{m}"
line = next(l for l in open(f"{d}/bench.log") if l.startswith('{"metric"'))
b = json.loads(line)
summ = open(f"{d}/summary.md").read()
cfg = b["config"]
out = [f"# r2 {m}: routed bench line + kernel profile (1x MI355X)\n",
       f"Command: `MODEL={m} CONVS={cfg['global_batch']} STEPS={b['steps']} bash scripts/gpu_model_bench.sh` "
       "(bench.py with random-init weights of the true architecture; both tiers served by this model on one GPU; "
       "hybrid router, semantic cache on, GPU MiniLM encoder).  Run 1 tunes GEMM plans, run 2 is profiled "
       "(rocprofv3 --kernel-trace --stats; 1 warm-up + the timed steps).\n",
       "| metric | value |", "|---|---|"]
for k in ("value", "ms_per_step", "p50_latency_ms", "p90_latency_ms", "ttft_ms_p50", "avg_decode_batch",
          "engine_decode_tok_s", "prefix_cache_hit_rate", "small_tier_share", "requests"):
    out.append(f"| {k} | {b.get(k)} |")
out.append(f"| engine_time_split_s | {b.get('engine_time_split_s')} |")
out.append(f"| router_encoder | {b.get('router_encoder')} |")
out += ["", "Bench line (unprofiled run):", "", "```", line.strip(), "```", "", "## Kernel time (profiled run)", "", summ]
open(f"profiles/r2_{m}_bench_kernels.md", "w").write("\n".join(out) + "\n")
print(f"profiles/r2_{m}_bench_kernels.md")
