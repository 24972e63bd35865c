#!/bin/bash
# Same-box A/B of the round-4 knobs at the 1-GPU (F) and per-rank (R) shapes: base, the hidden head's
# backward on the split kernels at every batch, PX at every batch, base again; then the PX tests.
set -o pipefail
TAG=${1:-r04d}
O=gpurun_out/$TAG
mkdir -p $O
R="--envs 512 --batch-size 2048 --steps 5 --warmup 2 --no-cpu-baseline"
F="--steps 4 --warmup 2 --no-cpu-baseline"
for P in R F; do
  timeout -k 10 300 python -u bench.py ${!P} > $O/${P}_base.json 2>> $O/bench.err || exit $?
  PPOX_HEAD_BWD_SPLIT_MIN=0 timeout -k 10 300 python -u bench.py ${!P} > $O/${P}_hbwd.json 2>> $O/bench.err || exit $?
  PPOX_PX_MIN=0 timeout -k 10 300 python -u bench.py ${!P} > $O/${P}_pxall.json 2>> $O/bench.err || exit $?
  timeout -k 10 300 python -u bench.py ${!P} > $O/${P}_base2.json 2>> $O/bench.err || exit $?
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_px_gpu.py \
    > $O/tests.log 2>&1 || exit $?
echo done > $O/DONE
