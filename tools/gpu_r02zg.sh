set -o pipefail
O=gpurun_out/r02zg; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { echo FAIL; grep -E "^FAILED|Error" $O/t.log | head -20; tail -3 $O/t.log; exit 1; }
for s in 1 0; do
  PPOX_BWD_STREAMS=$s timeout -k 10 300 python bench.py --algo rnd --envs 1024 --batch-size 16384 --steps 2 --warmup 1 --no-cpu-baseline > $O/rnd_$s.json 2>>$O/err.log || exit 1
  grep -o '"ms_per_step": [0-9.]*' $O/rnd_$s.json | sed "s/^/rnd streams=$s /" >> $O/ab.txt
  PPOX_BWD_STREAMS=$s timeout -k 10 300 python bench.py --envs 512 --batch-size 2048 --steps 3 --warmup 1 --no-cpu-baseline > $O/rank_$s.json 2>>$O/err.log || exit 1
  grep -o '"ms_per_step": [0-9.]*' $O/rank_$s.json | sed "s/^/rank streams=$s /" >> $O/ab.txt
done
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/full.json 2>>$O/err.log || exit 1
grep -o '"ms_per_step": [0-9.]*' $O/full.json | sed "s/^/full streams=1 /" >> $O/ab.txt
echo done
