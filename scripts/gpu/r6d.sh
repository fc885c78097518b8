# round 6: packed-dot GEMV + skinny_epi at B = 1-16, tgemm grouped raster probe
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6d
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 MB_DECODE_C=2048 MB_TEMP=0.8
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tgemm_gpu.py tests/test_kernels_gpu.py -k "gemv or skinny or raster" > gpurun_out/r6d/tests.log 2>&1 || { tail -30 gpurun_out/r6d/tests.log; exit 1; }
tail -2 gpurun_out/r6d/tests.log
MB_DECODE_B=1,2,4,8,16 DLLM_VERBOSE=1 timeout -k 10 500 python3 scripts/microbench.py --what decode > gpurun_out/r6d/tiny.log 2>&1 || { tail -20 gpurun_out/r6d/tiny.log; exit 1; }
grep '^{' gpurun_out/r6d/tiny.log | cut -c1-200
MB_DECODE_B=1,8 DLLM_VERBOSE=1 timeout -k 10 600 python3 scripts/microbench.py --model llama-3-8b --what decode > gpurun_out/r6d/l8b.log 2>&1 || { tail -20 gpurun_out/r6d/l8b.log; exit 1; }
grep '^{' gpurun_out/r6d/l8b.log | cut -c1-200
timeout -k 10 400 python -u scripts/exp/raster_probe.py > gpurun_out/r6d/raster.jsonl 2> gpurun_out/r6d/raster.err || { tail -20 gpurun_out/r6d/raster.err; exit 1; }
cut -c1-600 gpurun_out/r6d/raster.jsonl
