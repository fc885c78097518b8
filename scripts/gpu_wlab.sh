#!/bin/bash
# Round-4 decode-GEMM probes at M = 320: cold (rotated weight copies) vs warm (one weight copy
# re-read by every launch), and loader-only probes that move one operand (W-ONLY / A-ONLY)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/wlab
for N in ${LAB_NS:-2048}; do
  timeout -k 10 240 ./labbin2/gemmlab 320 $N - notg > gpurun_out/wlab/cold2_n$N.jsonl 2>&1 || exit $?
  LAB_COPIES=1 timeout -k 10 240 ./labbin2/gemmlab 320 $N - notg > gpurun_out/wlab/warm2_n$N.jsonl 2>&1 || exit $?
done
echo wlab ok
