set -o pipefail
O=gpurun_out/r02zb; mkdir -p $O
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { echo FAIL; grep -E "^FAILED|Error" $O/t.log | head -20; tail -3 $O/t.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/rz -o run --output-format csv -- \
    python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
cp /tmp/rz/*kernel_stats* $O/kernel_stats.csv
timeout -k 10 200 python tools/fc_bench.py 4096 > $O/fc4k.jsonl 2>&1 || exit 1
timeout -k 10 200 python tools/fc_bench.py 8192 > $O/fc8k.jsonl 2>&1 || exit 1
echo done
