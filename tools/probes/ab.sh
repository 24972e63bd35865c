#!/bin/bash
# A/B of variant libraries on the bench (dev tool): tools/probes/ab.sh TAG VARIANT [VARIANT...]
# Runs the kernel tests selected by TESTK (default: conv2_dgrad) on each variant, then base, each
# variant, base again at the 1-GPU (F) and per-rank (R) shapes (PHASES, default "F R"; I: the
# PPO_ICM per-rank shape).  Writes gpurun_out/ab_TAG/.
set -o pipefail
TAG=$1; shift
O=gpurun_out/ab_$TAG; mkdir -p $O
R="--envs 512 --batch-size 2048 --steps 5 --warmup 2 --no-cpu-baseline"
F="--steps 4 --warmup 2 --no-cpu-baseline"
I="--algo icm --envs 512 --batch-size 2048 --steps 3 --warmup 1 --no-cpu-baseline"
for V in "$@"; do
  PPOX_LIB=tools/variants/$V/libppox.so timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q \
      -k "${TESTK:-conv2_dgrad}" --timeout 200 --timeout-method thread > $O/tests_$V.log 2>&1 || exit $?
done
for P in ${PHASES:-F R}; do
  timeout -k 10 200 python bench.py ${!P} > $O/${P}_base.json 2>>$O/e || exit $?
  for V in "$@"; do
    PPOX_LIB=tools/variants/$V/libppox.so timeout -k 10 200 python bench.py ${!P} > $O/${P}_$V.json 2>>$O/e || exit $?
  done
  timeout -k 10 200 python bench.py ${!P} > $O/${P}_base2.json 2>>$O/e || exit $?
done
