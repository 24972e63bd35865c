#!/bin/bash
# conv kernel timings (tools/probes/conv_bench.py) for the main library and each variant named on the command line.
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for v in base "$@"; do
  if [ $v = base ]; then L=""; else L=tools/variants/$v/libppox.so; fi
  if [ -z "$L" ]; then timeout -k 10 200 python -u tools/probes/conv_bench.py 16384 > gpurun_out/$TAG/$v.log 2>&1 || exit $?
  else timeout -k 10 200 python -u tools/probes/conv_bench.py 16384 $L > gpurun_out/$TAG/$v.log 2>&1 || exit $?; fi
done
