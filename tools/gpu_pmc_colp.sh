# FETCH/WRITE passes for the persistent conv2 dgrad kernel (bench workload, one epoch)
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O=gpurun_out/r02c2; mkdir -p $O
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "colp_kernel" -d /tmp/colp-$C -o run \
      --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --epochs 1 --no-cpu-baseline \
      > $O/pmc_$C.log 2>&1 || exit $?
  cp /tmp/colp-$C/*counter_collection* $O/pmc_$C.csv
done
python3 tools/pmc_summary.py $O/pmc_FETCH_SIZE.csv $O/pmc_WRITE_SIZE.csv $O/pmc_summary.json > $O/pmc_summary.txt || exit 1
echo done
