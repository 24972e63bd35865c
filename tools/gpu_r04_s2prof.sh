#!/bin/bash
# Round-4 second-session profiles (run via gpurun): tools/gpu_profile.sh (rocprofv3 stats, by-grid, timeline,
# PMC FETCH/WRITE), then the SQ counter passes of the split kernels (tools/kernel_pmc.sh).
set -o pipefail
TAG=${1:-r04s2prof}
tools/gpu_profile.sh $TAG || exit $?
tools/kernel_pmc.sh ${TAG}_sq "sgemm|wgrad|colp|fwd1|dconv" bench.py --steps 1 --warmup 0 --epochs 1 --no-cpu-baseline \
    || exit $?
echo done > gpurun_out/$TAG/DONE2
