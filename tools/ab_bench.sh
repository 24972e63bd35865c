#!/bin/bash
# Same-box A/B of bench.py (run via gpurun): the main library and each variant library named on the command
# line (tools/variants/NAME/libppox.so, loaded through PPOX_LIB), the 1-GPU line and the per-rank shape, two
# rounds.  Writes gpurun_out/TAG/NAME_{F,R}{1,2}.json.
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
for rnd in 1 2; do
  for v in base "$@"; do
    if [ $v = base ]; then L=""; else L=tools/variants/$v/libppox.so; fi
    PPOX_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 > $O/${v}_F$rnd.json 2>> $O/err.log || exit $?
    PPOX_LIB=$L timeout -k 10 300 python -u bench.py --envs 512 --batch-size 2048 --steps 5 --warmup 2 --no-cpu-baseline \
        > $O/${v}_R$rnd.json 2>> $O/err.log || exit $?
  done
done
