#!/bin/bash
# Current routing harness (src/tests/routing_chatbot_tester.py protocol: each query set is ONE growing
# conversation per experiment, reference per-query + summary CSVs) with the reference's model pair on
# one MI355X: phi3-mini small tier, Llama-3-8B large tier (data/topologies/reference_models_1gpu.json).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/harness_ref; mkdir -p $OUT
export DLLM_GEMM_PLANS=$OUT/gemm_plans.json
for qs in ${QUERY_SETS:-general_knowledge technical_coding personal_health}; do
  timeout -k 10 900 python3 -m distributed_llm_amd.bench.harness --query-set $qs \
    --pools distributed_llm_amd/data/topologies/reference_models_1gpu.json \
    --strategies ${STRATEGIES:-token heuristic semantic hybrid perf} --cache-modes off --thresholds ${THRESHOLDS:-400} \
    --output-csv $OUT/benchmark_results.csv --output-per-query-csv $OUT/benchmark_per_query.csv --resume \
    > $OUT/$qs.log 2>&1 || { echo "$qs failed rc=$?"; tail -20 $OUT/$qs.log; exit 1; }
  echo "$qs done"
done
