set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6s
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python3 -u scripts/exp/insitu_probe.py 448 480 512 > gpurun_out/r6s/insitu.txt 2>&1 || { tail -20 gpurun_out/r6s/insitu.txt; exit 1; }
cat gpurun_out/r6s/insitu.txt
