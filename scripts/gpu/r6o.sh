# round 6: full GPU test suite + smoke on the current tree (prefill core autotuned by default)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6o
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r6o/gpu_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r6o/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6o/smoke.log 2>&1 || { tail -20 gpurun_out/r6o/smoke.log; exit 1; }
tail -2 gpurun_out/r6o/smoke.log
