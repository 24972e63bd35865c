# ICM: parity tests + bench + kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r02x; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x -k "icm or ICM or c4" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { echo FAIL; grep -E "^FAILED|Error" $O/t.log | head -20; tail -3 $O/t.log; exit 1; }
timeout -k 10 300 python bench.py --algo icm --envs 512 --batch-size 2048 --steps 2 --warmup 1 --no-cpu-baseline > $O/icm.json 2>$O/icm.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/icm -o run --output-format csv -- \
    python3 $R/bench.py --algo icm --envs 512 --batch-size 2048 --steps 1 --warmup 1 --no-cpu-baseline > $O/icm_prof.log 2>&1 || exit 1
cp /tmp/icm/*kernel_stats* $O/icm_kernel_stats.csv
echo done
