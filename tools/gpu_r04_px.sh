#!/bin/bash
# Round-4 PX check on the GPU box: the PX tests + the touched kernel / product tests, then the bench
# line and the per-rank shape with PX off and on (same box).  Writes gpurun_out/TAG/.
set -o pipefail
TAG=${1:-r04px}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_px_gpu.py \
    tests/test_kernels_gpu.py -k "px or pack_all or h1p or fc_ or conv3 or sg2 or split_conv or explicit or relu_bits" \
    > $O/tests.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_product_gpu.py -k "cnn" \
    >> $O/tests.log 2>&1 || exit $?
for PX in 0 1; do
  PPOX_PX=$PX timeout -k 10 300 python -u bench.py --envs 512 --batch-size 2048 --steps 5 --warmup 2 --no-cpu-baseline \
      > $O/bench_rank_px$PX.json 2>> $O/bench.err || exit $?
done
for PX in 0 1; do
  PPOX_PX=$PX timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline > $O/bench_px$PX.json 2>> $O/bench.err || exit $?
done
echo done > $O/DONE
