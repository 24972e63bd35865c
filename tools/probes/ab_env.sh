#!/bin/bash
# A/B of environment settings at the per-rank (R) and 1-GPU (F) shapes (dev tool):
#   tools/probes/ab_env.sh TAG SHAPES "VAR=value ..." ["VAR=value ..." ...]   (SHAPES: R, F or "R F")
# runs base, each setting, base again per shape.  Writes gpurun_out/abenv_TAG/.
set -o pipefail
TAG=$1; SHAPES=$2; shift 2
O=gpurun_out/abenv_$TAG; mkdir -p $O
R="--envs 512 --batch-size 2048 --steps 5 --warmup 2 --no-cpu-baseline"
F="--steps 4 --warmup 2 --no-cpu-baseline"
for P in $SHAPES; do
  timeout -k 10 200 python bench.py ${!P} > $O/${P}_base.json 2>>$O/e || exit $?
  i=0
  for SETTING in "$@"; do
    i=$((i+1))
    env $SETTING timeout -k 10 200 python bench.py ${!P} > $O/${P}_v$i.json 2>>$O/e || exit $?
  done
  timeout -k 10 200 python bench.py ${!P} > $O/${P}_base2.json 2>>$O/e || exit $?
done
