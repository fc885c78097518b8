#!/bin/bash
# Reference-style routing benchmark on 1 GPU (BASELINE config 2): each query set replayed as ONE
# growing conversation per (strategy, cache mode, threshold), reference per-query + summary CSVs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/harness; mkdir -p $OUT
export DLLM_GEMM_PLANS=$OUT/gemm_plans.json
for qs in ${QUERY_SETS:-general_knowledge technical_coding personal_health}; do
  timeout -k 10 900 python3 -m distributed_llm_amd.bench.harness --query-set $qs --pools gpu \
    --strategies token heuristic semantic hybrid perf --cache-modes off on --thresholds ${THRESHOLDS:-200 400 1000} \
    --output-csv $OUT/benchmark_results.csv --output-per-query-csv $OUT/benchmark_per_query.csv --resume \
    > $OUT/$qs.log 2>&1 || { echo "$qs failed rc=$?"; tail -20 $OUT/$qs.log; exit 1; }
  echo "$qs done"; tail -2 $OUT/$qs.log
done
