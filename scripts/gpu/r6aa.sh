# round 6: 16-row loader-wave tgemm tiles for batch <= 16: numerics (every epilogue, split-K), then
# TinyLlama / Llama-3-8B decode steps at B = 1-16 with the in-situ autotune
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6aa
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 MB_DECODE_C=2048 MB_TEMP=0.8
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_tgemm_gpu.py > gpurun_out/r6aa/tgemm_tests.log 2>&1 || { tail -30 gpurun_out/r6aa/tgemm_tests.log; exit 1; }
tail -1 gpurun_out/r6aa/tgemm_tests.log
MB_DECODE_B=1,2,4,8,16 DLLM_VERBOSE=1 timeout -k 10 500 python3 scripts/microbench.py --what decode > gpurun_out/r6aa/tiny.log 2>&1 || { tail -20 gpurun_out/r6aa/tiny.log; exit 1; }
grep '^{' gpurun_out/r6aa/tiny.log | cut -c1-110
MB_DECODE_B=1,4,8 DLLM_VERBOSE=1 timeout -k 10 600 python3 scripts/microbench.py --model llama-3-8b --what decode > gpurun_out/r6aa/l8b.log 2>&1 || { tail -20 gpurun_out/r6aa/l8b.log; exit 1; }
grep '^{' gpurun_out/r6aa/l8b.log | cut -c1-110
grep -c "(16, 128" gpurun_out/r6aa/tiny.log gpurun_out/r6aa/l8b.log || true
