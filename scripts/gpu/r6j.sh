# round 6 (review item 3): batch 2-8 GEMV with the grid capped on wide projections: numerics under
# three grid policies, same-process probe (off vs default), then TinyLlama / Llama-3-8B decode steps
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6j
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 MB_DECODE_C=2048 MB_TEMP=0.8
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tgemm_gpu.py tests/test_kernels_gpu.py -k "gemv" > gpurun_out/r6j/gemv_tests.log 2>&1 || { tail -30 gpurun_out/r6j/gemv_tests.log; exit 1; }
tail -2 gpurun_out/r6j/gemv_tests.log
DLLM_GEMV_GRIDS="1:0:0,512:4:8192" timeout -k 10 400 python3 -u scripts/exp/gemv_probe.py 2 4 8 > gpurun_out/r6j/gemv_probe.jsonl 2> gpurun_out/r6j/gemv_probe.err || { tail -20 gpurun_out/r6j/gemv_probe.err; exit 1; }
wc -l gpurun_out/r6j/gemv_probe.jsonl
MB_DECODE_B=1,2,4,8,16 DLLM_VERBOSE=1 timeout -k 10 500 python3 scripts/microbench.py --what decode > gpurun_out/r6j/tiny.log 2>&1 || { tail -20 gpurun_out/r6j/tiny.log; exit 1; }
grep '^{' gpurun_out/r6j/tiny.log | cut -c1-200
MB_DECODE_B=1,2,4,8 DLLM_VERBOSE=1 timeout -k 10 600 python3 scripts/microbench.py --model llama-3-8b --what decode > gpurun_out/r6j/l8b.log 2>&1 || { tail -20 gpurun_out/r6j/l8b.log; exit 1; }
grep '^{' gpurun_out/r6j/l8b.log | cut -c1-200
