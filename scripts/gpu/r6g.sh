# round 6 (review item 6): one-GPU rehearsals of the multi-GPU bench paths with FULL-depth models and
# decode graphs ON: the driver's default at N = 2 / 4 (config-2 replicas) and config 3 (1B | 8B pools)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6g
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 DLLM_REHEARSE_ONE_GPU=1 OMP_NUM_THREADS=2 MASTER_ADDR=127.0.0.1
run() {  # name, timeout, nproc, bench args...
  local name=$1 t=$2 n=$3; shift 3
  timeout -k 10 $t python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + RANDOM % 1000)) bench.py --gpus $n "$@" > gpurun_out/r6g/$name.log 2>&1 \
    || { echo "$name failed"; tail -30 gpurun_out/r6g/$name.log; return 1; }
  grep '^{"metric"' gpurun_out/r6g/$name.log > gpurun_out/r6g/$name.json
  python3 -c "
import json; d=json.load(open('gpurun_out/r6g/$name.json'))
print('$name', d['value'], d['baseline_config'], d['config']['parallelism'], 'init', d['init_s'], 'startup', d['startup_s'], 'per_gpu', d.get('per_gpu_tok_s'), 'rehearsal', d.get('rehearsal_one_gpu'))"
}
run rep2 420 2 --steps 3 --warmup 1 --convs 128 --kv-gb 16 && \
run rep4 480 4 --steps 3 --warmup 1 --convs 64 --kv-gb 8 && \
run cfg3 540 2 --baseline-config 3 --steps 3 --warmup 1 --convs 64 --kv-gb 8
