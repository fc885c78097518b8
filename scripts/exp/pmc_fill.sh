#!/bin/bash
# Side-by-side fill-path counters of hipBLASLt's 256x256 kernel and tgemm's 256x256 cores on the
# Llama-3-8B down shape at 4K rows (M 4096, N 4096, K 14336): one rocprofv3 --pmc pass per counter
# group (SQ issue/stall, TA/TD/TCP fill path, TCC L2), kernel-trace only, each under its own timeout.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp PYTHONPATH=.
out=gpurun_out/pmc_fill
mkdir -p $out
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
FILL="TA_TA_BUSY_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE"
L2="TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_TAG_STALL_sum"
for v in "blas blas" "pp 256,256,4,1,1,8,1,0,0,32" "k64 256,256,2,1,1,8" "m32 256,256,2,1,1,8,1,0,0,64,32"; do
  set -- $v
  for g in SQ FILL L2; do
    timeout -s KILL 90 rocprofv3 --pmc ${!g} --output-format csv -d $out/$1_$g -o run -- \
      python3 scripts/exp/tg_one.py 4096 4096 14336 $2 5 > $out/$1_$g.log 2>&1 || { echo "pmc $1 $g failed"; tail -5 $out/$1_$g.log; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob, collections, json
rows = {}
for f in glob.glob("gpurun_out/pmc_fill/*/**/run_counter_collection.csv", recursive=True) + \
         glob.glob("gpurun_out/pmc_fill/*/run_counter_collection.csv"):
    tag = f.split("/")[2].split("_")[0]
    agg = rows.setdefault(tag, collections.defaultdict(float)); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "tgemm" not in k and "Cijk" not in k:
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
for tag, agg in sorted(rows.items()):
    print(json.dumps({"kernel": tag, **{k: v for k, v in sorted(agg.items())}}))
PY
