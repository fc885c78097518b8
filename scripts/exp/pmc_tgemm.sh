mkdir -p gpurun_out/pmc && export PYTHONPATH=. && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmc/p1 -o run -- python scripts/exp/tg_one.py 4096 4096 14336 256,256,4,1,1,8,1,0,0,32 5 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmc/p2 -o run -- python scripts/exp/tg_one.py 4096 4096 14336 256,256,2,1,1,8 5 && \
for d in p1 p2; do f=$(ls gpurun_out/pmc/$d/*/run_counter_collection.csv gpurun_out/pmc/$d/run_counter_collection.csv 2>/dev/null | head -1); python - "$f" "$d" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(float); n = collections.Counter()
for r in rows:
    if 'tgemm' not in r['Kernel_Name']: continue
    agg[r['Counter_Name']] += float(r['Counter_Value']); n[r['Counter_Name']] += 1
print(sys.argv[2], {k: round(v / max(1, n[k])) for k, v in sorted(agg.items())})
PY
done
