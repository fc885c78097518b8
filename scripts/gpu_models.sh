#!/bin/bash
# True-shape model-family checks on one MI355X: fp32-reference + graph==eager tests, then a
# decode-step microbench per family.  Every GPU step has its own time limit; the script stops at
# the first crash / timeout (no retries).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/test_models_gpu.py -x -v --timeout 600 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/models_gpu.log 2>&1
rc=$?; echo "models pytest rc=$rc"; tail -15 gpurun_out/models_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
for m in ${MODELS:-llama-3-8b}; do
  MB_DECODE_B=${MB_DECODE_B:-1,64,256} MB_DECODE_C=${MB_DECODE_C:-2048} timeout -k 10 600 \
    python -u scripts/microbench.py --model $m --what decode > gpurun_out/decode_$m.jsonl 2>&1
  rc=$?; echo "decode $m rc=$rc"; tail -4 gpurun_out/decode_$m.jsonl
  if [ $rc -ne 0 ]; then exit $rc; fi
done
exit 0
