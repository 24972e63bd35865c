#!/bin/bash
# Per-kernel stats of the per-rank shape (512 envs, minibatch 2048) for the in-tree library and
# each variant (dev tool): tools/rank_stats.sh TAG [VARIANT...] -> gpurun_out/rs_TAG/<name>_kernel_stats.csv
# (ALGO=icm / rnd: that algorithm's per-rank shape)
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/rs_$TAG; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for V in base "$@"; do
  L=""; [ "$V" != base ] && L=$R/tools/variants/$V/libppox.so
  PPOX_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/rs-$TAG-$V -o run --output-format csv -- \
      python3 $R/bench.py --algo ${ALGO:-ppo} --envs 512 --batch-size 2048 --steps 2 --warmup 1 --no-cpu-baseline > $O/${V}_bench.json \
      2> $O/${V}.err || exit $?
  find /tmp/rs-$TAG-$V -name "*kernel_stats.csv" -exec cp {} $O/${V}_kernel_stats.csv \; || exit 1
done
