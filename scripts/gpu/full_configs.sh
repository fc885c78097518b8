#!/bin/bash
# BASELINE configs 5 and 4 at their TRUE model sizes, launched exactly as the driver launches the
# 8-GPU pools bench, but with all 8 ranks sharing ONE MI355X (DLLM_REHEARSE_ONE_GPU=1: gloo groups,
# one-shot IPC all-reduce for the TP pool).  Config 5: Llama-3.2-1B x4 | Mixtral-8x7B TP=4 (~103 GB
# of weights on the card); config 4: Llama-3-8B x4 | Llama-3-70B TP=4 (~205 GB).  Throughput here
# is 8 processes time-slicing one GPU: this proves the configurations run, it measures nothing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/fullcfg
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLLM_REHEARSE_ONE_GPU=1 DLLM_AUTOTUNE=0 OMP_NUM_THREADS=2 \
  MASTER_ADDR=127.0.0.1 DLLM_EMBEDDER=hash
( while true; do sleep 45; echo "tick $(date +%T) $(tail -c 200 $O/cfg*.log 2>/dev/null | tail -1 | cut -c1-120)"; done ) &
TICK=$!
trap "kill $TICK 2>/dev/null" EXIT
for cfg in ${CFGS:-5 4}; do
  timeout -k 10 ${CFG_TIMEOUT:-600} python -m torch.distributed.run --nnodes=1 --nproc-per-node=8 --master-addr 127.0.0.1 \
    --master-port $((29500 + cfg)) bench.py --gpus 8 --topology pools --baseline-config $cfg --steps 2 --warmup 0 \
    --convs 2 --kv-gb 2 --small-new 16 --large-new 24 --greedy --no-graphs --strategy hybrid > $O/cfg$cfg.log 2>&1
  rc=$?; echo "config $cfg rc=$rc"; grep '^{"metric"' $O/cfg$cfg.log | cut -c1-400
  [ $rc -ne 0 ] && { tail -30 $O/cfg$cfg.log | cut -c1-300; exit $rc; }
done
exit 0
