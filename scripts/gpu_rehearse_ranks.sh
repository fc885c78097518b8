#!/bin/bash
# Rehearse the driver's multi-rank bench command on a one-GPU box: N ranks under torch.distributed.run,
# all on GPU 0 with gloo collectives (bench.py DLLM_REHEARSE_ONE_GPU=1), small KV pools.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLLM_REHEARSE_ONE_GPU=1
mkdir -p gpurun_out/rehearse
for n in ${RANKS:-2 4}; do
  timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --steps 2 --warmup 1 --convs 128 --kv-gb 16 \
    > gpurun_out/rehearse/n$n.log 2>&1 || { echo "n=$n failed rc=$?"; tail -30 gpurun_out/rehearse/n$n.log; exit 1; }
  echo "n=$n: $(grep -o '"value": [0-9.]*, "unit"[^}]*"n_gpus": [0-9]*' gpurun_out/rehearse/n$n.log) $(grep -o '"rehearsal_one_gpu": true' gpurun_out/rehearse/n$n.log)"
done
