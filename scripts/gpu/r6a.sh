set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6a
export TMPDIR=/tmp
timeout -k 10 400 python scripts/cache_scorer_bench.py > gpurun_out/r6a/cache_scorer.jsonl 2> gpurun_out/r6a/cache_scorer.err || { tail -20 gpurun_out/r6a/cache_scorer.err; exit 1; }
cat gpurun_out/r6a/cache_scorer.jsonl
timeout -k 10 60 rocprofv3 -L > gpurun_out/r6a/counters.txt 2>&1 || true
PROF_TAG=r6a_prof STEPS=6 bash scripts/gpu/profile.sh
