# Round-2 split-f16 measurements: bench line, rocprof kernel stats, PMC passes of the conv2
# dgrad and the fc GEMMs, the per-rank-shape line.
set -o pipefail
O=gpurun_out/r02h; mkdir -p $O
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 500 python bench.py > $O/bench.json 2>$O/bench.err || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/rf -o run --output-format csv -- \
    python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
cp /tmp/rf/*kernel_stats* $O/kernel_stats.csv
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "colp_kernel|SgRows<" -d /tmp/pmc-$C -o run \
      --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --epochs 1 --no-cpu-baseline \
      > $O/pmc_$C.log 2>&1 || exit 1
  cp /tmp/pmc-$C/*counter_collection* $O/pmc_$C.csv
done
python3 tools/pmc_summary.py $O/pmc_FETCH_SIZE.csv $O/pmc_WRITE_SIZE.csv $O/pmc_summary.json > $O/pmc_summary.txt || exit 1
timeout -k 10 300 python bench.py --envs 512 --batch-size 2048 --steps 3 --warmup 1 --no-cpu-baseline > $O/rank.json 2>>$O/err.log || exit 1
echo done
