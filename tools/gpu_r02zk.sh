set -o pipefail
O=gpurun_out/r02zk; mkdir -p $O
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
for s in 8192 0; do
  PPOX_FC_SPLIT_MIN=$s timeout -k 10 300 python bench.py --envs 512 --batch-size 2048 --steps 3 --warmup 1 --no-cpu-baseline > $O/rank_$s.json 2>>$O/err.log || exit 1
  grep -o '"ms_per_step": [0-9.]*' $O/rank_$s.json | sed "s/^/rank fc_split_min=$s /" >> $O/ab.txt
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/rz -o run --output-format csv -- \
    python3 $R/bench.py --envs 512 --batch-size 2048 --steps 1 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
cp /tmp/rz/*kernel_stats* $O/rank_kernel_stats.csv
echo done
