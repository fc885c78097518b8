# round 6 (review item 3): where a TinyLlama decode step's time goes at B = 2 / 4 / 8 (sampled rows,
# C = 2048): one tuning run writes the plan file, then one kernel-trace run per batch size replays it
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6k
export HSA_ENABLE_IPC_MODE_LEGACY=0 MB_DECODE_C=2048 MB_TEMP=0.8 DLLM_GEMM_PLANS=$R/gpurun_out/r6k/plans.json
cd $R && MB_DECODE_B=2,4,8 DLLM_VERBOSE=1 timeout -k 10 400 python3 scripts/microbench.py --what decode > gpurun_out/r6k/tune.log 2>&1 || { tail -20 gpurun_out/r6k/tune.log; exit 1; }
grep '^{' gpurun_out/r6k/tune.log | cut -c1-160
cd /tmp && export TMPDIR=/tmp
for B in 2 4 8; do
  MB_DECODE_B=$B timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6k/b$B -o p -- python3 $R/scripts/microbench.py --what decode > $R/gpurun_out/r6k/b$B.log 2>&1 || { tail -20 $R/gpurun_out/r6k/b$B.log; exit 1; }
  grep '^{' $R/gpurun_out/r6k/b$B.log | cut -c1-160
done
