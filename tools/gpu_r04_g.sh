#!/bin/bash
# PPO_ICM per-rank with the data-parallel branches forced on: host profile and host lag.
set -o pipefail
TAG=${1:-r04g}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python3 tools/host_profile.py 512 2048 icm dist > $O/host_profile_icm_dist.txt 2>&1 || exit $?
timeout -k 10 300 python3 tools/host_profile.py 512 2048 icm > $O/host_profile_icm.txt 2>&1 || exit $?
echo done > $O/DONE
