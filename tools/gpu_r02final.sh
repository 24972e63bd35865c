# Round-2 final measurements: GPU suite, the bench line, its rocprof kernel stats, PMC passes of
# the dominant kernel, the other configs' lines.
set -o pipefail
O=gpurun_out/r02final; mkdir -p $O
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { echo FAIL; grep -E "^FAILED|Error" $O/t.log | head -20; tail -3 $O/t.log; exit 1; }
timeout -k 10 500 python bench.py > $O/bench.json 2>$O/bench.err || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/rf -o run --output-format csv -- \
    python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
cp /tmp/rf/*kernel_stats* $O/kernel_stats.csv
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "colp_kernel" -d /tmp/colp-$C -o run \
      --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --epochs 1 --no-cpu-baseline \
      > $O/pmc_$C.log 2>&1 || exit 1
  cp /tmp/colp-$C/*counter_collection* $O/pmc_$C.csv
done
python3 tools/pmc_summary.py $O/pmc_FETCH_SIZE.csv $O/pmc_WRITE_SIZE.csv $O/pmc_summary.json > $O/pmc_summary.txt || exit 1
timeout -k 10 300 python bench.py --envs 512 --batch-size 2048 --steps 3 --warmup 1 --no-cpu-baseline > $O/rank.json 2>>$O/err.log || exit 1
timeout -k 10 300 python bench.py --algo icm --envs 512 --batch-size 2048 --steps 2 --warmup 1 --no-cpu-baseline > $O/icm.json 2>>$O/err.log || exit 1
timeout -k 10 300 python bench.py --algo rnd --envs 1024 --batch-size 16384 --steps 2 --warmup 1 --no-cpu-baseline > $O/rnd.json 2>>$O/err.log || exit 1
echo done
