#!/bin/bash
# Round-4 decode-GEMM probes: cold (rotated weight copies) vs warm (one copy) weights, M = 320
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/wlab
for N in ${LAB_NS:-2048 11264}; do
  timeout -k 10 240 ./labbin2/gemmlab 320 $N - > gpurun_out/wlab/cold_n$N.jsonl 2>&1 || exit $?
  LAB_COPIES=1 timeout -k 10 240 ./labbin2/gemmlab 320 $N - > gpurun_out/wlab/warm_n$N.jsonl 2>&1 || exit $?
done
echo wlab ok
