#!/bin/bash
# PMC passes over one decode-GEMM lab variant (scripts/exp/gemmlab.hip), one rocprofv3 run per
# counter group (gfx950: <= 8 SQ counters per pass).  Usage: gemm_pmc.sh M N VARIANT_SUBSTRING
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
M=$1; N=$2; V=$3; TAG=${4:-pmc}
mkdir -p gpurun_out/$TAG
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_BUSY_avr"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --stats -d gpurun_out/$TAG/p$i -o run -- \
      scripts/exp/bin/gemmlab $M $N "$V" notg > gpurun_out/$TAG/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/$TAG/p$i.log; exit 1; }
done
echo done
