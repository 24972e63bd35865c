#!/bin/bash
# ICM sharded-path fix check + per-rank host lag (one-rank RCCL forced on) + the per-rank profile.
set -o pipefail
TAG=${1:-r04e}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_icm_gpu.py \
    tests/test_c4_gpu.py > $O/tests.log 2>&1 || exit $?
A="--envs 512 --batch-size 2048 --no-cpu-baseline"
timeout -k 10 300 python -u bench.py --algo icm $A --steps 3 --warmup 1 --force-dist > $O/bench_icm_dist.json 2>> $O/bench.err || exit $?
timeout -k 10 300 python -u bench.py --algo icm $A --steps 3 --warmup 1 > $O/bench_icm.json 2>> $O/bench.err || exit $?
timeout -k 10 300 python -u bench.py $A --steps 5 --warmup 2 --force-dist > $O/bench_rank_dist.json 2>> $O/bench.err || exit $?
for V in "ppo x" "ppo dist" "icm dist"; do
  set -- $V
  timeout -k 10 300 python -u tools/host_lag.py 512 2048 $1 $2 > $O/host_lag_$1_$2.txt 2>> $O/bench.err || exit $?
done
tools/gpu_r04_rank.sh ${TAG}_rank || exit $?
echo done > $O/DONE
