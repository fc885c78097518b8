# round 6: tgemm 32x32x16 plans (numerics, timing vs 16x16x32 and hipBLASLt), fill-path counters,
# batch-8 decode kernel table
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6b
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tgemm_gpu.py > gpurun_out/r6b/tgemm_tests.log 2>&1 || { tail -30 gpurun_out/r6b/tgemm_tests.log; exit 1; }
tail -2 gpurun_out/r6b/tgemm_tests.log
timeout -k 10 400 python -u scripts/exp/m32_probe.py > gpurun_out/r6b/m32_probe.jsonl 2> gpurun_out/r6b/m32_probe.err || { tail -20 gpurun_out/r6b/m32_probe.err; exit 1; }
cut -c1-400 gpurun_out/r6b/m32_probe.jsonl
bash scripts/exp/pmc_fill.sh > gpurun_out/r6b/pmc_fill.jsonl 2>&1 || { tail -20 gpurun_out/r6b/pmc_fill.jsonl; exit 1; }
cat gpurun_out/r6b/pmc_fill.jsonl
MB_DECODE_B=8 MB_DECODE_C=2048 MB_TEMP=0.8 DLLM_VERBOSE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6b/b8 -o p --output-format csv -- python3 scripts/microbench.py --what decode > gpurun_out/r6b/b8.log 2>&1 || { tail -20 gpurun_out/r6b/b8.log; exit 1; }
grep '^{' gpurun_out/r6b/b8.log | cut -c1-300
f=$(find gpurun_out/r6b/b8 -name "*kernel_stats.csv" | head -1)
python3 scripts/prof_summary.py "$f" 30 > gpurun_out/r6b/b8_kernels.md && head -34 gpurun_out/r6b/b8_kernels.md
find gpurun_out/r6b/b8 -name "*trace*" -delete
