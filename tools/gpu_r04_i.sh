#!/bin/bash
# ICM sharded-path host work (native scatter, zeroing in the pair entry): ICM / C4 / RCCL tests, then
# per-rank host lag (ICM one process / forced dist, PPO) and the ICM bench lines.
set -o pipefail
TAG=${1:-r04i}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_icm_gpu.py \
    tests/test_c4_gpu.py tests/test_rccl_gpu.py > $O/tests.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/event_probe.py 200 > $O/event_probe.txt 2>> $O/err || exit $?
timeout -k 10 300 python -u tools/host_lag.py 512 2048 icm x > $O/host_lag_icm.txt 2>> $O/err || exit $?
timeout -k 10 300 python -u tools/host_lag.py 512 2048 icm dist > $O/host_lag_icm_dist.txt 2>> $O/err || exit $?
timeout -k 10 300 python -u tools/host_lag.py 512 2048 ppo x > $O/host_lag_ppo.txt 2>> $O/err || exit $?
A="--algo icm --envs 512 --batch-size 2048 --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 python -u bench.py $A --force-dist > $O/bench_icm_dist.json 2>> $O/err || exit $?
timeout -k 10 300 python -u bench.py $A > $O/bench_icm.json 2>> $O/err || exit $?
echo done > $O/DONE
R="--envs 512 --batch-size 2048 --steps 5 --warmup 2 --no-cpu-baseline"
for k in 1 2; do
  timeout -k 10 300 python -u bench.py $R > $O/R_base$k.json 2>> $O/err || exit $?
  PPOX_W2P_MIN_PER=16 timeout -k 10 300 python -u bench.py $R > $O/R_w2p16_$k.json 2>> $O/err || exit $?
  PPOX_W2P_MIN_PER=32 timeout -k 10 300 python -u bench.py $R > $O/R_w2p32_$k.json 2>> $O/err || exit $?
  PPOX_FORK_MERGE=1 timeout -k 10 300 python -u bench.py $R > $O/R_merge_$k.json 2>> $O/err || exit $?
done
echo done > $O/DONE2
