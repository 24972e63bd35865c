set -o pipefail
O=gpurun_out/r02zq; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { echo FAIL; grep -E "^FAILED|Error" $O/t.log | head -20; tail -3 $O/t.log; exit 1; }
timeout -k 10 300 python tools/host_lag.py 512 2048 > $O/host_lag.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --envs 512 --batch-size 2048 --steps 3 --warmup 1 --no-cpu-baseline > $O/rank.json 2>>$O/err.log || exit 1
grep -o '"ms_per_step": [0-9.]*' $O/rank.json | sed "s/^/rank /" >> $O/ab.txt
echo done
