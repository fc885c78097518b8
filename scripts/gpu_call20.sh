#!/bin/bash
# Host-side CPU budget of the flagship window: per-thread CPU share (routing driver vs the
# engine step loop) and a cProfile of the driver thread.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/cpu20
mkdir -p $O
export DLLM_GEMM_PLANS=$O/gemm_plans.json
DLLM_THREAD_CPU=1 DLLM_SYNC_LOG=1 DLLM_DRIVER_PROFILE=$O/driver.prof \
  timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > $O/run.log 2>&1 \
  || { echo "bench failed"; tail -30 $O/run.log; exit 1; }
tail -1 $O/run.log
python3 -c "
import pstats; s = pstats.Stats('$O/driver.prof'); s.sort_stats('tottime').print_stats(40)
s.sort_stats('cumulative').print_stats(40)" > $O/driver_prof.txt 2>&1
head -60 $O/driver_prof.txt
