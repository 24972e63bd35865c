# kernel stats of the ICM (per-rank shape) and RND (C3) iterations
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r02v; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/icm -o run --output-format csv -- \
    python3 $R/bench.py --algo icm --envs 512 --batch-size 2048 --steps 1 --warmup 1 --no-cpu-baseline > $O/icm.log 2>&1 || exit 1
cp /tmp/icm/*kernel_stats* $O/icm_kernel_stats.csv
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/rnd -o run --output-format csv -- \
    python3 $R/bench.py --algo rnd --envs 1024 --batch-size 16384 --steps 1 --warmup 1 --no-cpu-baseline > $O/rnd.log 2>&1 || exit 1
cp /tmp/rnd/*kernel_stats* $O/rnd_kernel_stats.csv
echo done
