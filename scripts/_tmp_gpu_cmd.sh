set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/gn
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemv or engine or graph or tinyllama" > gpurun_out/gn/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/gn/pytest.log; [ $rc -eq 0 ] || exit $rc
export DLLM_GEMM_PLANS=gpurun_out/gn/plans.json MB_DECODE_B=1,2,4,8 MB_DECODE_C=1024
timeout -k 10 400 python3 scripts/microbench.py --what decode > gpurun_out/gn/fused.log 2>&1 || exit $?
DLLM_FUSED_NORM=0 timeout -k 10 400 python3 scripts/microbench.py --what decode > gpurun_out/gn/unfused.log 2>&1 || exit $?
grep decode_step gpurun_out/gn/fused.log gpurun_out/gn/unfused.log | cut -c1-160
