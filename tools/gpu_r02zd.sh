set -o pipefail
O=gpurun_out/r02zd; mkdir -p $O
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { echo FAIL; grep -E "^FAILED|Error" $O/t.log | head -20; tail -3 $O/t.log; exit 1; }
timeout -k 10 300 python bench.py --algo rnd --envs 1024 --batch-size 16384 --steps 2 --warmup 1 --no-cpu-baseline > $O/rnd.json 2>$O/rnd.err || exit 1
timeout -k 10 300 python bench.py --envs 512 --batch-size 2048 --steps 3 --warmup 1 --no-cpu-baseline > $O/rank.json 2>$O/rank.err || exit 1
timeout -k 10 400 python bench.py --steps 2 --warmup 1 > $O/bench.json 2>$O/bench.err || exit 1
echo done
