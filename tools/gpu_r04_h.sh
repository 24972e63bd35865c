#!/bin/bash
# Graph replay vs eager at 2,048 rows for capture-order / head variants (tools/graph_probe.py), then a
# kernel trace of the best-guess variant's replay.
set -o pipefail
TAG=${1:-r04h}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
for V in base late hbwd late_hbwd; do
  E=""
  case $V in late) E="PPOX_FORK_LATE=1";; hbwd) E="PPOX_HEAD_BWD_SPLIT_MIN=0";; late_hbwd) E="PPOX_FORK_LATE=1 PPOX_HEAD_BWD_SPLIT_MIN=0";; esac
  env $E timeout -k 10 200 python3 -u tools/graph_probe.py 2048 60 > $O/probe_$V.log 2>&1 || exit $?
done
export TMPDIR=/tmp
cd /tmp
PPOX_FORK_LATE=1 PPOX_HEAD_BWD_SPLIT_MIN=0 timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/$TAG-g -o run \
    --output-format csv -- python3 $R/tools/graph_probe.py 2048 40 graph > $O/trace_graph.log 2>&1 || exit $?
T=$(find /tmp/$TAG-g -name "*kernel_trace.csv" | head -n 1)
python3 $R/tools/timeline.py $T 3 > $O/timeline_graph_late_hbwd.txt || exit $?
echo done > $O/DONE
