#!/bin/bash
# Round-4 profiles (run via gpurun): tools/gpu_profile.sh (rocprofv3 stats, by-grid, timeline, PMC
# FETCH/WRITE), then the SQ counter passes of the split kernels (tools/kernel_pmc.sh).
set -o pipefail
TAG=${1:-r04prof}
tools/gpu_profile.sh $TAG || exit $?
tools/kernel_pmc.sh ${TAG}_sq "sgemm|wgrad|colp|fwd1" bench.py --steps 1 --warmup 0 --epochs 1 --no-cpu-baseline \
    || exit $?
timeout -k 10 300 python3 tools/host_profile.py 512 2048 icm dist > gpurun_out/$TAG/host_profile_icm_dist.txt 2>&1 \
    || exit $?
echo done > gpurun_out/$TAG/DONE2
