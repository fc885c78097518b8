set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/wl
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/wl/pytest_eng.log 2>&1; rc=$?; tail -3 gpurun_out/wl/pytest_eng.log; [ $rc -eq 0 ] || exit $rc
STEPS=8 WARMUP=2 bash scripts/ab_args.sh "" || exit $?
DLLM_ATTN_WORKLIST=0 STEPS=8 WARMUP=2 bash scripts/ab_args.sh "" || exit $?
STEPS=8 WARMUP=2 bash scripts/ab_args.sh ""
