#!/bin/bash
# rocprofv3 kernel stats + one-minibatch timelines of the 1-GPU line and the per-rank shape with the
# env knob KNOB (default PPOX_PX) at 0 and 1 (dev tool): tools/px_ab_prof.sh TAG [KNOB]
set -o pipefail
TAG=$1; KNOB=${2:-PPOX_PX}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for V in 0 1; do
  for SHAPE in big rank; do
    if [ $SHAPE = big ]; then A="--steps 1 --warmup 1"; else A="--envs 512 --batch-size 2048 --steps 2 --warmup 1"; fi
    env $KNOB=$V true  # (the knob reaches the profiled program through the environment below)
    export $KNOB=$V
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/$TAG-$V-$SHAPE -o run --output-format csv -- \
        python3 $R/bench.py $A --no-cpu-baseline > $O/${SHAPE}_$V.json 2> $O/${SHAPE}_$V.err || exit $?
    find /tmp/$TAG-$V-$SHAPE -name "*kernel_stats.csv" -exec cp {} $O/${SHAPE}_${V}_kernel_stats.csv \; || exit 1
    T=$(find /tmp/$TAG-$V-$SHAPE -name "*kernel_trace.csv" | head -1)
    python3 $R/tools/timeline.py $T 3 > $O/${SHAPE}_${V}_timeline.txt || exit $?
  done
done
echo done > $O/DONE
