# round 6: small-batch fused-epilogue MFMA GEMM (skinny_epi) numerics + decode steps at B = 1-16
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6c
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 MB_DECODE_C=2048 MB_TEMP=0.8
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tgemm_gpu.py -k "skinny_epi" > gpurun_out/r6c/ske_tests.log 2>&1 || { tail -30 gpurun_out/r6c/ske_tests.log; exit 1; }
tail -2 gpurun_out/r6c/ske_tests.log
MB_DECODE_B=1,2,4,8,16 DLLM_VERBOSE=1 timeout -k 10 500 python3 scripts/microbench.py --what decode > gpurun_out/r6c/tiny.log 2>&1 || { tail -20 gpurun_out/r6c/tiny.log; exit 1; }
grep '^{' gpurun_out/r6c/tiny.log | cut -c1-200
grep "core" gpurun_out/r6c/tiny.log | grep -E "gemm M=(1|2|4|8|16) " | cut -c1-300
MB_DECODE_B=1,8 DLLM_VERBOSE=1 timeout -k 10 600 python3 scripts/microbench.py --model llama-3-8b --what decode > gpurun_out/r6c/l8b.log 2>&1 || { tail -20 gpurun_out/r6c/l8b.log; exit 1; }
grep '^{' gpurun_out/r6c/l8b.log | cut -c1-200
