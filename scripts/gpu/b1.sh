#!/bin/bash
# Small-batch decode step times (sampled rows, C = 2048) and a kernel table of the TinyLlama B = 1 replay.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 MB_DECODE_C=2048 MB_TEMP=0.8
tag=${B1_TAG:-b1}
mkdir -p gpurun_out/$tag
MB_DECODE_B=${B1_BS:-1,2,4,8} timeout -k 10 400 python3 scripts/microbench.py --what decode > gpurun_out/$tag/tiny.log 2>&1 || exit $?
grep '^{' gpurun_out/$tag/tiny.log | cut -c1-200
MB_DECODE_B=1 timeout -k 10 500 python3 scripts/microbench.py --model llama-3-8b --what decode > gpurun_out/$tag/l8b.log 2>&1 || exit $?
grep '^{' gpurun_out/$tag/l8b.log | cut -c1-200
if [ -n "$B1_PROF" ]; then
  MB_DECODE_B=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag/prof -o p --output-format csv -- \
    python3 scripts/microbench.py --what decode > gpurun_out/$tag/prof.log 2>&1 || exit $?
  f=$(find gpurun_out/$tag/prof -name "*kernel_stats.csv" | head -1)
  python3 scripts/prof_summary.py "$f" 40 > gpurun_out/$tag/kernels.md && head -45 gpurun_out/$tag/kernels.md
  find gpurun_out/$tag/prof -name "*trace*" -delete
fi
