#!/bin/bash
# GPU-box profiling recipe (run via gpurun from the repo root).  Writes small
# summaries under gpurun_out/; full traces stay in /tmp on the box.
# Usage: tools/gpu_profile.sh TAG
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/$TAG/bench.json.log 2>&1 || exit $?
timeout -k 10 200 python tools/gae_sweep.py > gpurun_out/$TAG/gae_sweep.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/$TAG-stats -o run --output-format csv -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/stats.log 2>&1 || exit $?
cp /tmp/$TAG-stats/*stats* gpurun_out/$TAG/
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "wgrad_kernel|gae|gemm|split_kernel|col_kernel|colp_kernel|wgrad_reduce" -d /tmp/$TAG-$C -o run \
      --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --epochs 1 --no-cpu-baseline \
      > gpurun_out/$TAG/pmc_$C.log 2>&1 || exit $?
  cp /tmp/$TAG-$C/*counter_collection* gpurun_out/$TAG/pmc_$C.csv
done
python3 tools/pmc_summary.py gpurun_out/$TAG/pmc_FETCH_SIZE.csv gpurun_out/$TAG/pmc_WRITE_SIZE.csv \
    gpurun_out/$TAG/pmc_summary.json > gpurun_out/$TAG/pmc_summary.txt || exit $?
timeout -k 10 200 python tools/conv_bench.py > gpurun_out/$TAG/conv_bench.jsonl 2>&1 || exit $?
echo done > gpurun_out/$TAG/DONE
