#!/bin/bash
# Round-4 check: new / touched GPU tests, then the PX A/B bench pair at both shapes (same box).
set -o pipefail
TAG=${1:-r04b}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_px_gpu.py \
    tests/test_es_dist.py tests/test_es.py \
    tests/test_kernels_gpu.py -k "px or pack_all or h1p or fc_ or conv3 or sg2 or split_conv or explicit or relu_bits or big_minibatch or es_ or conv2_dgrad" \
    > $O/tests.log 2>&1 || exit $?
for PX in 0 1; do
  PPOX_PX=$PX timeout -k 10 300 python -u bench.py --envs 512 --batch-size 2048 --steps 5 --warmup 2 --no-cpu-baseline \
      > $O/bench_rank_px$PX.json 2>> $O/bench.err || exit $?
  PPOX_PX=$PX timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline > $O/bench_px$PX.json 2>> $O/bench.err || exit $?
done
echo done > $O/DONE
