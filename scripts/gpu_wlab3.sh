#!/bin/bash
# Shared vs private activation tiles in the decode-GEMM lab (M = 512): A-PRIVATE variants give every
# n-tile its own replica of A, so no two CUs read the same activation line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/wlab
timeout -k 10 200 ./labbin2/gemmlab 512 0 A-PRIVATE notg > gpurun_out/wlab/priv_m512.jsonl 2>&1 || exit $?
timeout -k 10 200 ./labbin2/gemmlab 512 0 "rg<64,64,2x2+4,st8,S1> ROT" notg > gpurun_out/wlab/shared_m512.jsonl 2>&1 || exit $?
echo wlab3 ok
