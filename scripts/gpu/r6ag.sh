# round 6 final tree: TinyLlama / Llama-3-8B decode steps at B = 1-16 (in-situ autotune, qkv_post v2)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6ag
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 MB_DECODE_C=2048 MB_TEMP=0.8
MB_DECODE_B=1,2,4,8,16 DLLM_VERBOSE=1 timeout -k 10 500 python3 scripts/microbench.py --what decode > gpurun_out/r6ag/tiny.log 2>&1 || { tail -20 gpurun_out/r6ag/tiny.log; exit 1; }
grep '^{' gpurun_out/r6ag/tiny.log | cut -c1-110
MB_DECODE_B=1,4,8 DLLM_VERBOSE=1 timeout -k 10 600 python3 scripts/microbench.py --model llama-3-8b --what decode > gpurun_out/r6ag/l8b.log 2>&1 || { tail -20 gpurun_out/r6ag/l8b.log; exit 1; }
grep '^{' gpurun_out/r6ag/l8b.log | cut -c1-110
