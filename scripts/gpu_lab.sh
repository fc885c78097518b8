#!/bin/bash
# Decode-GEMM lab probes (prebuilt in labbin/ by hipcc here): per-CU intake ceilings and the GEMM
# variant table at the serving batch sizes.  Each probe has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/lab
timeout -k 10 120 ./labbin/intake > gpurun_out/lab/intake.jsonl 2>&1 || exit $?
timeout -k 10 120 ./labbin/intake rows > gpurun_out/lab/intake_rows.jsonl 2>&1 || exit $?
for M in ${LAB_MS:-320 512}; do
  timeout -k 10 300 ./labbin/gemmlab $M > gpurun_out/lab/gemmlab_m$M.jsonl 2>&1 || exit $?
done
echo lab ok
