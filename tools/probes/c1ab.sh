#!/bin/bash
# conv1 forward timings (tools/probes/conv1_bench.py) for the main library and each variant named on the command line.
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for v in base "$@"; do
  if [ $v = base ]; then L=""; else L=tools/variants/$v/libppox.so; fi
  PPOX_LIB=$L timeout -k 10 200 python -u tools/probes/conv1_bench.py 4096 16384 > gpurun_out/$TAG/$v.log 2>&1 || exit $?
done
