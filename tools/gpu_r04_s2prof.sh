#!/bin/bash
# Round-4 second-session profiles (run via gpurun): tools/gpu_profile.sh (rocprofv3 stats, by-grid, timeline,
# PMC FETCH/WRITE), then the SQ counter passes of the split kernels (tools/kernel_pmc.sh).
set -o pipefail
TAG=${1:-r04s2prof}
tools/gpu_profile.sh $TAG || exit $?
tools/kernel_pmc.sh ${TAG}_sq "sgemm|wgrad|colp|fwd1|dconv|fcd_kernel" bench.py --steps 1 --warmup 0 --epochs 1 --no-cpu-baseline \
    || exit $?
echo done > gpurun_out/$TAG/DONE2
# PPO_ICM with the data-parallel branches over a one-rank RCCL communicator, twice (its spread across boxes)
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --algo icm --envs 512 --batch-size 2048 --steps 3 --warmup 1 --no-cpu-baseline \
      --force-dist > gpurun_out/$TAG/bench_icm_dist_$r.json 2>> gpurun_out/$TAG/icm.err || exit $?
done
echo done > gpurun_out/$TAG/DONE3
