set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/pb1 gpurun_out/pb8
export TMPDIR=/tmp
export DLLM_GEMM_PLANS=gpurun_out/pb1/plans.json MB_KV_GB=8 MB_MAX_SEQS=16 MB_DECODE_C=2048
MB_DECODE_B=1 timeout -k 10 300 python3 scripts/microbench.py --what decode > gpurun_out/pb1/tune.log 2>&1 || exit $?
MB_DECODE_B=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pb1 -o b1 --output-format csv -- python3 scripts/microbench.py --what decode > gpurun_out/pb1/run.log 2>&1 || exit $?
MB_DECODE_B=8 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pb8 -o b8 --output-format csv -- python3 scripts/microbench.py --what decode > gpurun_out/pb8/run.log 2>&1 || exit $?
for b in 1 8; do f=$(find gpurun_out/pb$b -name "*kernel_trace.csv" | head -1); python3 scripts/replay_trace.py "$f" > gpurun_out/pb$b/replay.md; rm -f "$f"; cat gpurun_out/pb$b/replay.md | head -30; done
cat gpurun_out/pb1/tune.log | grep decode_step
