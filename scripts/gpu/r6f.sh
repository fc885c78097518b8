# round 6: pruned tgemm build (GPU numerics + refusal), then the driver command with the KV run-miss breakdown
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6f
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tgemm_gpu.py > gpurun_out/r6f/tgemm_tests.log 2>&1 || { tail -30 gpurun_out/r6f/tgemm_tests.log; exit 1; }
tail -2 gpurun_out/r6f/tgemm_tests.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6f/bench.log 2>&1 || { tail -20 gpurun_out/r6f/bench.log; exit 1; }
grep '^{' gpurun_out/r6f/bench.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print(d['value'], d['prefix_cache_hit_rate'], d['kv_block_placement'], d['startup_s'])"
