set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/gv
export DLLM_GEMM_PLANS=gpurun_out/gv/plans.json MB_DECODE_B=1,4,16 MB_DECODE_C=1024,4096
timeout -k 10 400 python3 scripts/microbench.py --what decode > gpurun_out/gv/a.log 2>&1 || exit $?
DLLM_ATTN_WL_MIN_BS=1 timeout -k 10 400 python3 scripts/microbench.py --what decode > gpurun_out/gv/b.log 2>&1 || exit $?
DLLM_ATTN_WAVES=4 timeout -k 10 400 python3 scripts/microbench.py --what decode > gpurun_out/gv/c.log 2>&1 || exit $?
DLLM_ATTN_WL_MIN_BS=1 DLLM_ATTN_WAVES=4 timeout -k 10 400 python3 scripts/microbench.py --what decode > gpurun_out/gv/d.log 2>&1 || exit $?
for f in a b c d; do echo == $f; grep decode_step gpurun_out/gv/$f.log | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print(d['B'], d['C'], d['ms'])"; done
