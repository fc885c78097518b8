#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pf
export DLLM_VERBOSE=1
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/pf/tuned.log 2>&1 || exit $?
grep "gemm prefill" gpurun_out/pf/tuned.log | cut -c1-200
tail -1 gpurun_out/pf/tuned.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('prefill-tuned', d['value'], d['engine_time_split_s']['t_prefill_s'])"
DLLM_PREFILL_TUNE=0 timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/pf/untuned.log 2>&1 || exit $?
tail -1 gpurun_out/pf/untuned.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('untuned', d['value'], d['engine_time_split_s']['t_prefill_s'])"
