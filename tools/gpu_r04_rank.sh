#!/bin/bash
# Round-4 per-rank-shape profile (run via gpurun): kernel trace of the per-rank bench (512 envs,
# minibatch 2048) -> one minibatch's timeline + stats; then tools/graph_probe.py at 2,048 rows under
# --kernel-trace, eager and captured (the epoch-graph question), each with its timeline.
set -o pipefail
TAG=${1:-r04rank}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
export TMPDIR=/tmp
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/$TAG-rank -o run --output-format csv -- \
    python3 $R/bench.py --envs 512 --batch-size 2048 --steps 2 --warmup 1 --no-cpu-baseline \
    > $O/bench_rank.json 2> $O/rank.err || exit $?
T=$(find /tmp/$TAG-rank -name "*kernel_trace.csv" | head -n 1)
find /tmp/$TAG-rank -name "*kernel_stats.csv" -exec cp {} $O/rank_kernel_stats.csv \; || exit 1
python3 $R/tools/timeline.py $T 3 > $O/timeline_rank_minibatch.txt || exit $?
python3 $R/tools/gaps.py $T 5 ${LAST_MS:-260} > $O/gaps_rank.txt || exit $?
for V in eager graph; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/$TAG-$V -o run --output-format csv -- \
      python3 $R/tools/graph_probe.py 2048 40 $V > $O/probe_$V.log 2>&1 || exit $?
  T=$(find /tmp/$TAG-$V -name "*kernel_trace.csv" | head -n 1)
  python3 $R/tools/timeline.py $T 3 > $O/probe_timeline_$V.txt || exit $?
done
echo done > $O/DONE
