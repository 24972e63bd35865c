# bench lines (PPO 1-GPU, per-rank shape, RND C3, ICM C4 per rank, ES C5) + per-rank kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r02l; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > $O/bench.json 2>$O/bench.err || exit 1
timeout -k 10 300 python bench.py --envs 512 --batch-size 2048 --steps 3 --warmup 1 --no-cpu-baseline > $O/rank.json 2>$O/rank.err || exit 1
timeout -k 10 300 python bench.py --algo rnd --envs 1024 --batch-size 16384 --steps 2 --warmup 1 --no-cpu-baseline > $O/rnd.json 2>$O/rnd.err || exit 1
timeout -k 10 300 python bench.py --algo icm --envs 512 --batch-size 2048 --steps 2 --warmup 1 --no-cpu-baseline > $O/icm.json 2>$O/icm.err || exit 1
timeout -k 10 300 python bench.py --algo es --steps 2 --warmup 1 > $O/es.json 2>$O/es.err || exit 1
timeout -k 10 200 python tools/host_lag.py 512 2048 > $O/host_lag.txt 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/rk -o run --output-format csv -- \
    python3 $R/bench.py --envs 512 --batch-size 2048 --steps 2 --warmup 1 --no-cpu-baseline > $O/rank_stats.log 2>&1 || exit 1
cp /tmp/rk/*stats* $O/
echo done
