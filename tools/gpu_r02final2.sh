# Round-2 closing refresh: full GPU suite, bench line, rocprof kernel stats, PMC passes of the
# split kernels (training-size launches), per-rank shape (+ its kernel stats), RND / ICM / ES lines.
set -o pipefail
O=gpurun_out/r02final2; mkdir -p $O
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { echo FAIL; grep -E "^FAILED|Error" $O/t.log | head -20; tail -3 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 500 python bench.py > $O/bench.json 2>$O/bench.err || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/rf -o run --output-format csv -- \
    python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
cp /tmp/rf/*kernel_stats* $O/kernel_stats.csv
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "colp_kernel|sgemm_kernel|wgrad_split_kernel|fwd1_split" \
      -d /tmp/pmc-$C -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --epochs 1 --no-cpu-baseline \
      > $O/pmc_$C.log 2>&1 || exit 1
  cp /tmp/pmc-$C/*counter_collection* $O/pmc_$C.csv
done
python3 tools/pmc_summary.py $O/pmc_FETCH_SIZE.csv $O/pmc_WRITE_SIZE.csv $O/pmc_summary.json > $O/pmc_summary.txt || exit 1
timeout -k 10 300 python bench.py --envs 512 --batch-size 2048 --steps 3 --warmup 1 --no-cpu-baseline > $O/rank.json 2>>$O/err.log || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/rr -o run --output-format csv -- \
    python3 $R/bench.py --envs 512 --batch-size 2048 --steps 1 --warmup 1 --no-cpu-baseline > $O/prof_rank.log 2>&1 || exit 1
cp /tmp/rr/*kernel_stats* $O/rank_kernel_stats.csv
timeout -k 10 300 python bench.py --algo icm --envs 512 --batch-size 2048 --steps 2 --warmup 1 --no-cpu-baseline > $O/icm.json 2>>$O/err.log || exit 1
timeout -k 10 300 python bench.py --algo rnd --envs 1024 --batch-size 16384 --steps 2 --warmup 1 --no-cpu-baseline > $O/rnd.json 2>>$O/err.log || exit 1
timeout -k 10 300 python bench.py --algo es --steps 3 --warmup 1 --no-cpu-baseline > $O/es.json 2>>$O/err.log || exit 1
timeout -k 10 200 python tools/conv_bench.py 16384 > $O/conv_bench.jsonl 2>>$O/err.log || exit 1
echo done
