#!/bin/bash
# PX threshold A/B with the direct conv forwards (run via gpurun): bench line and per-rank shape with the
# default PPOX_PX_MIN (8,192 rows) and with PX at every batch (collect included).  Writes gpurun_out/TAG/.
set -o pipefail
TAG=${1:-r04s2b}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit $?
PPOX_PX_MIN=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_px0.json 2>> $O/bench.err || exit $?
timeout -k 10 300 python -u bench.py --envs 512 --batch-size 2048 --steps 5 --warmup 2 --no-cpu-baseline \
    > $O/bench_rank_shape.json 2>> $O/bench.err || exit $?
PPOX_PX_MIN=0 timeout -k 10 300 python -u bench.py --envs 512 --batch-size 2048 --steps 5 --warmup 2 \
    --no-cpu-baseline > $O/bench_rank_shape_px0.json 2>> $O/bench.err || exit $?
echo done > $O/DONE
