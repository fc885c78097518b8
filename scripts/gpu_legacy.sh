#!/bin/bash
# The reference's published protocol with its own model pair (phi3-mini + Llama-3-8B) on one MI355X
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/legacy_r4
mkdir -p $O
export DLLM_GEMM_PLANS=$O/gemm_plans.json
timeout -k 10 900 python3 -u scripts/legacy_ref_models.py $O > $O/run.log 2>&1 || { tail -30 $O/run.log; exit 1; }
python3 scripts/legacy_ref_report.py $O > $O/report.md 2>&1 || { tail -20 $O/report.md; exit 1; }
cat $O/report.md | head -60
