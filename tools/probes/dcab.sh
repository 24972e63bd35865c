#!/bin/bash
# dconv A/B (dev): the dconv parity tests, then tools/dconv_bench.py with the main library and each
# variant named on the command line (tools/variants/NAME/libppox.so).  Writes gpurun_out/TAG/.
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_dconv_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/$TAG/tests.log 2>&1 || exit $?
for v in base "$@"; do
  if [ $v = base ]; then L=ppo-exploration_amd/libppox.so; else L=tools/variants/$v/libppox.so; fi
  PPOX_LIB=$L timeout -k 10 120 python -u tools/dconv_bench.py 2048 16384 > gpurun_out/$TAG/$v.log 2>&1 || exit $?
done
