#!/bin/bash
# Round-4 second-session check (run via gpurun): the GPU suite, then the bench line and the per-rank shape,
# the direct conv forwards on (the default) and off (PPOX_DCONV2=0 PPOX_DCONV3=0) back to back.
set -o pipefail
TAG=${1:-r04s2}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit $?
PPOX_DCONV2=0 PPOX_DCONV3=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_nodc.json 2>> $O/bench.err || exit $?
timeout -k 10 300 python -u bench.py --envs 512 --batch-size 2048 --steps 5 --warmup 2 --no-cpu-baseline \
    > $O/bench_rank_shape.json 2>> $O/bench.err || exit $?
PPOX_DCONV2=0 PPOX_DCONV3=0 timeout -k 10 300 python -u bench.py --envs 512 --batch-size 2048 --steps 5 --warmup 2 \
    --no-cpu-baseline > $O/bench_rank_shape_nodc.json 2>> $O/bench.err || exit $?
echo done > $O/DONE
