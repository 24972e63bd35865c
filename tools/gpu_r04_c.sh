#!/bin/bash
# Round-4 check: new / touched GPU tests, then A/Bs on one box: the wide fc tiles (base) against the
# 64-column tiles (variant nb64), and PX off / on, at the 1-GPU (F) and per-rank (R) shapes.
set -o pipefail
TAG=${1:-r04c}
O=gpurun_out/$TAG
mkdir -p $O
R="--envs 512 --batch-size 2048 --steps 5 --warmup 2 --no-cpu-baseline"
F="--steps 4 --warmup 2 --no-cpu-baseline"
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_px_gpu.py \
    tests/test_kernels_gpu.py -k "px or pack_all or h1p or fc_ or conv3 or sg2 or split_conv or explicit or relu_bits or big_minibatch or head_hidden or split_f16" \
    > $O/tests.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_product_gpu.py -k "cnn" \
    >> $O/tests.log 2>&1 || exit $?
for P in F R; do
  timeout -k 10 300 python -u bench.py ${!P} > $O/${P}_base.json 2>> $O/bench.err || exit $?
  PPOX_LIB=tools/variants/nb64/libppox.so timeout -k 10 300 python -u bench.py ${!P} > $O/${P}_nb64.json 2>> $O/bench.err || exit $?
  PPOX_PX=0 timeout -k 10 300 python -u bench.py ${!P} > $O/${P}_px0.json 2>> $O/bench.err || exit $?
  timeout -k 10 300 python -u bench.py ${!P} > $O/${P}_base2.json 2>> $O/bench.err || exit $?
done
echo done > $O/DONE
