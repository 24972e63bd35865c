# per-rank shape (512 envs x 128, minibatch 2048): bench line, kernel stats, host lag
set -o pipefail
O=gpurun_out/r02i2; mkdir -p $O
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 300 python bench.py --envs 512 --batch-size 2048 --steps 3 --warmup 1 --no-cpu-baseline > $O/rank.json 2>$O/err.log || exit 1
timeout -k 10 300 python tools/host_lag.py 512 2048 > $O/host_lag.txt 2>>$O/err.log || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/rr -o run --output-format csv -- \
    python3 $R/bench.py --envs 512 --batch-size 2048 --steps 1 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
cp /tmp/rr/*kernel_stats* $O/kernel_stats.csv
echo done
