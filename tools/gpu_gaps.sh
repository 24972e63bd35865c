#!/bin/bash
# GPU idle-gap analysis of one bench iteration (dev tool): kernel trace under rocprofv3, then
# tools/gaps.py over the last iteration.  Usage: tools/gpu_gaps.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/gaps_$TAG
export TMPDIR=/tmp
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/gaps-$TAG -o run --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline "$@" > $O/bench.json 2> $O/err || exit $?
T=$(find /tmp/gaps-$TAG -name "*kernel_trace.csv" | head -n 1)
python3 $R/tools/gaps.py $T 50 ${LAST_MS:-1300} > $O/gaps.txt || exit $?
python3 $R/tools/timeline.py $T 3 > $O/timeline.txt || exit $?
