# L2 (TCC) hit / miss of the 256 x 256 tgemm core vs hipBLASLt on one prefill shape (one pass each)
mkdir -p gpurun_out/pmc2 && export PYTHONPATH=. && \
for v in "pp 256,256,4,1,1,8,1,0,0,32" "k64 256,256,2,1,1,8" "blas blas"; do set -- $v; \
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum --output-format csv -d gpurun_out/pmc2/$1 -o run -- python scripts/exp/tg_one.py 4096 4096 14336 $2 5 || exit 1; done && \
for d in pp k64 blas; do f=$(ls gpurun_out/pmc2/$d/*/run_counter_collection.csv gpurun_out/pmc2/$d/run_counter_collection.csv 2>/dev/null | head -1); python - "$f" "$d" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(float); n = collections.Counter(); names = collections.Counter()
for r in rows:
    k = r['Kernel_Name']
    if 'tgemm' not in k and 'Cijk' not in k: continue
    names[k[:60]] += 1
    agg[r['Counter_Name']] += float(r['Counter_Value']); n[r['Counter_Name']] += 1
hit, miss = agg['TCC_HIT_sum'], agg['TCC_MISS_sum']
print(sys.argv[2], dict(names), {k: round(v / max(1, n[k])) for k, v in sorted(agg.items())},
      'L2 hit rate %.3f' % (hit / max(1.0, hit + miss)))
PY
done
