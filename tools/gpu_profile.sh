#!/bin/bash
# GPU-box profiling recipe (run via gpurun from the repo root).  Writes small summaries under
# gpurun_out/TAG/; full traces stay in /tmp on the box.  Each GPU step has its own time limit and
# the steps are chained: the first failure ends the script.
# Usage: tools/gpu_profile.sh TAG
set -o pipefail
TAG=${1:-r03}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
export TMPDIR=/tmp
mkdir -p $O
cd /tmp
# the bench line + per-kernel stats of the same command
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/$TAG-stats -o run --output-format csv -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_under_rocprof.json 2> $O/stats.err || exit $?
find /tmp/$TAG-stats -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \; || exit 1
find /tmp/$TAG-stats -name "*kernel_trace.csv" -exec cp {} $O/kernel_trace.csv \; || exit 1
python3 $R/tools/trace_by_grid.py $O/kernel_trace.csv $O/kernel_by_grid.csv || exit $?
python3 $R/tools/timeline.py $O/kernel_trace.csv > $O/timeline_minibatch_16384.txt || exit $?
# HBM bytes per launch: FETCH_SIZE and WRITE_SIZE in separate passes (TCC counter slots)
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "wgrad|gae|gemm|split_kernel|colp_kernel|planes|dconv|fcd_kernel" \
      -d /tmp/$TAG-$C -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --epochs 1 \
      --no-cpu-baseline > $O/pmc_$C.log 2>&1 || exit $?
  find /tmp/$TAG-$C -name "*counter_collection.csv" -exec cp {} $O/pmc_$C.csv \; || exit 1
done
python3 $R/tools/pmc_summary.py $O/pmc_FETCH_SIZE.csv $O/pmc_WRITE_SIZE.csv $O/pmc_summary.json > $O/pmc_summary.txt \
    || exit $?
echo done > $O/DONE
