set -o pipefail
O=gpurun_out/r02zv; mkdir -p $O
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 300 python -u -m pytest tests/test_dist_gpu.py tests/test_product_gpu.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { echo FAIL; tail -3 $O/t.log; exit 1; }
for v in 8192 1000000 8192 1000000; do
  PPOX_BWD_SOLO_DGRAD2=$v timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/full_$v.json 2>>$O/err.log || exit 1
  python3 -c "
import json
d=json.loads(open('$O/full_$v.json').read().strip().splitlines()[-1]); r=d['roofline']
print('solo_min=$v', d['ms_per_step'], r['kernel'][:45], r['mean_us'], r['mean_us_isolated'], r['frac'])" >> $O/ab.txt
done
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/rf -o run --output-format csv -- \
    python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
cp /tmp/rf/*kernel_stats* $O/kernel_stats.csv
echo done
