# Kernel trace of the bench workload, per (kernel, grid size): the training-size launches' average
# of each kernel apart from its collect-size launches (rocprof --stats mixes them).
set -o pipefail
O=gpurun_out/r02final3; mkdir -p $O
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/rt -o run --output-format csv -- \
    python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
cp /tmp/rt/*kernel_stats* $O/kernel_stats.csv
python3 tools/trace_by_grid.py /tmp/rt/*kernel_trace.csv $O/kernel_by_grid.csv || exit 1
echo done
