set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/wl
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention or engine or graph" > gpurun_out/wl/pytest_attn.log 2>&1; rc=$?; tail -3 gpurun_out/wl/pytest_attn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/microbench.py --what attn_wl > gpurun_out/wl/attn_wl_pf.jsonl 2> gpurun_out/wl/attn_wl.err || { tail gpurun_out/wl/attn_wl.err; exit 1; }
DLLM_ATTN_BT_PREFETCH=0 timeout -k 10 300 python -u scripts/microbench.py --what attn_wl > gpurun_out/wl/attn_wl_nopf.jsonl 2> gpurun_out/wl/attn_wl.err || { tail gpurun_out/wl/attn_wl.err; exit 1; }
STEPS=8 WARMUP=2 bash scripts/ab_args.sh "" || exit $?
DLLM_ATTN_WORKLIST=0 STEPS=8 WARMUP=2 bash scripts/ab_args.sh "" || exit $?
DLLM_ATTN_BT_PREFETCH=0 STEPS=8 WARMUP=2 bash scripts/ab_args.sh ""
