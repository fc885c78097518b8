set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6a
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_router_gpu.py tests/test_kernel_resources.py > gpurun_out/r6a/tests.log 2>&1 || { tail -30 gpurun_out/r6a/tests.log; exit 1; }
tail -3 gpurun_out/r6a/tests.log
timeout -k 10 400 python scripts/cache_scorer_bench.py > gpurun_out/r6a/cache_scorer.jsonl 2> gpurun_out/r6a/cache_scorer.err || { tail -20 gpurun_out/r6a/cache_scorer.err; exit 1; }
cat gpurun_out/r6a/cache_scorer.jsonl
PROF_TAG=r6a_prof STEPS=6 bash scripts/gpu/profile.sh
