# round 6 (review item 3): batch 2-8 GEMV with a capped grid (X staged once per workgroup):
# numerics under three grid policies, then the same-process grid A/B per projection
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6h
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
true
true
DLLM_GEMV_GRIDS="1:0,256:4,256:8,512:4,256:16" timeout -k 10 500 python3 -u scripts/exp/gemv_probe.py 2 4 8 > gpurun_out/r6h/gemv_probe.jsonl 2> gpurun_out/r6h/gemv_probe.err || { tail -20 gpurun_out/r6h/gemv_probe.err; exit 1; }
wc -l gpurun_out/r6h/gemv_probe.jsonl
