set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u scripts/exp/two_stream.py > gpurun_out/two_stream.log 2>&1
rc=$?; tail -6 gpurun_out/two_stream.log; exit $rc
