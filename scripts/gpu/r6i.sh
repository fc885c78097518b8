# round 6 (review item 6): BASELINE config 4 at full depth, all 8 ranks rehearsed on ONE GPU
# (Llama-3-8B small replicas x4 + Llama-3-70B TP=4; gloo collectives, so the TP engines run eager):
# start-up time (weights + autotune) and per-rank peak device memory; then the config-2 replicas at
# N = 2 with decode graphs recorded in the JSON
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6i
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 DLLM_REHEARSE_ONE_GPU=1 OMP_NUM_THREADS=2 MASTER_ADDR=127.0.0.1
run() {  # name, timeout, nproc, bench args...
  local name=$1 t=$2 n=$3; shift 3
  timeout -k 10 $t python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + RANDOM % 1000)) bench.py --gpus $n "$@" > gpurun_out/r6i/$name.log 2>&1 \
    || { echo "$name failed"; tail -30 gpurun_out/r6i/$name.log; return 1; }
  grep '^{"metric"' gpurun_out/r6i/$name.log > gpurun_out/r6i/$name.json
  python3 -c "
import json; d=json.load(open('gpurun_out/r6i/$name.json'))
print('$name', d['value'], d['baseline_config'], d['config']['parallelism'], 'graphs', d['config'].get('decode_graphs'), 'init', d['init_s'], 'startup', d['startup_s'], 'mem', d.get('peak_device_mem_gb_by_rank'))"
}
rocm-smi --showmeminfo vram > gpurun_out/r6i/vram_before.txt 2>&1 || true
export DLLM_VERBOSE=1 && \
run cfg4 1000 8 --baseline-config 4 --steps 2 --warmup 0 --convs 8 --kv-gb 2 --small-new 32 --large-new 48
