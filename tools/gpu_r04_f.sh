#!/bin/bash
# PX df + conv1 whole-tile H1P epilogue: checks, then same-box A/B at the per-rank (R) and 1-GPU (F)
# shapes: base (both on), PPOX_PX_DF=0, the epi0 variant library (per-row conv1 epilogue).
set -o pipefail
TAG=${1:-r04f}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_px_gpu.py \
    tests/test_kernels_gpu.py -k "px or h1p or fc" > $O/tests.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_product_gpu.py \
    -k "cnn_train" > $O/tests_product.log 2>&1 || exit $?
R="--envs 512 --batch-size 2048 --steps 5 --warmup 2 --no-cpu-baseline"
F="--steps 4 --warmup 2 --no-cpu-baseline"
V=tools/variants/epi0/libppox.so
for P in R F; do
  for k in 1 2; do
    timeout -k 10 300 python -u bench.py ${!P} > $O/${P}_base$k.json 2>> $O/bench.err || exit $?
    PPOX_PX_DF=0 timeout -k 10 300 python -u bench.py ${!P} > $O/${P}_nodf$k.json 2>> $O/bench.err || exit $?
    PPOX_LIB=$V timeout -k 10 300 python -u bench.py ${!P} > $O/${P}_epi0$k.json 2>> $O/bench.err || exit $?
  done
done
echo done > $O/DONE
