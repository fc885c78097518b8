#!/bin/bash
# Rehearse `bench.py --topology pools` (tiers on disjoint GPU subsets, remote pools over the control /
# data planes) with N ranks sharing ONE GPU (DLLM_REHEARSE_ONE_GPU=1, gloo everywhere).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLLM_REHEARSE_ONE_GPU=1
mkdir -p gpurun_out/rehearse
for n in ${RANKS:-2}; do
  timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29600 + n)) bench.py --gpus $n --topology pools --steps 2 --warmup 1 --convs 32 --kv-gb 16 \
    --small-model ${SMALL:-llama-3.2-1b} --large-model ${LARGE:-llama-3-8b} \
    > gpurun_out/rehearse/pools_n$n.log 2>&1 || { echo "pools n=$n failed rc=$?"; tail -30 gpurun_out/rehearse/pools_n$n.log; exit 1; }
  echo "pools n=$n: $(grep -o '"value": [0-9.]*' gpurun_out/rehearse/pools_n$n.log) $(grep -o '"parallelism": "[^"]*"' gpurun_out/rehearse/pools_n$n.log)"
done
