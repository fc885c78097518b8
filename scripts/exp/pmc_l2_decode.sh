# L2 (TCC) hit rates of the flagship's decode GEMM plans at M = 480 (TinyLlama), one pass each
mkdir -p gpurun_out/pmc3 && export PYTHONPATH=. && \
for v in "gu 11264 2048 256,128,3,1,1,8,1,8" "qkv 2560 2048 64,128,4,1,1,8" "wo 2048 2048 64,64,2,1,2,4" "down 2048 5632 64,64,2,1,2,4,2"; do set -- $v; \
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum --output-format csv -d gpurun_out/pmc3/$1 -o run -- python scripts/exp/tg_one.py 480 $2 $3 $4 5 || exit 1; done && \
for d in gu qkv wo down; do f=$(ls gpurun_out/pmc3/$d/*/run_counter_collection.csv gpurun_out/pmc3/$d/run_counter_collection.csv 2>/dev/null | head -1); python - "$f" "$d" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(float); n = collections.Counter()
for r in rows:
    if 'tgemm' not in r['Kernel_Name']: continue
    agg[r['Counter_Name']] += float(r['Counter_Value']); n[r['Counter_Name']] += 1
hit, miss = agg['TCC_HIT_sum'], agg['TCC_MISS_sum']
print(sys.argv[2], {k: round(v / max(1, n[k])) for k, v in sorted(agg.items())}, 'L2 hit rate %.3f' % (hit / max(1.0, hit + miss)))
PY
done
