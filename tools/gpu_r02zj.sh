set -o pipefail
O=gpurun_out/r02zj; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { echo FAIL; grep -E "^FAILED|Error" $O/t.log | head -20; tail -3 $O/t.log; exit 1; }
for m in 8192 0; do
  PPOX_FC_SPLITK_MAX=$m timeout -k 10 300 python bench.py --envs 512 --batch-size 2048 --steps 3 --warmup 1 --no-cpu-baseline > $O/rank_$m.json 2>>$O/err.log || exit 1
  grep -o '"ms_per_step": [0-9.]*' $O/rank_$m.json | sed "s/^/rank splitk_max=$m /" >> $O/ab.txt
done
timeout -k 10 300 python bench.py --algo icm --envs 512 --batch-size 2048 --steps 2 --warmup 1 --no-cpu-baseline > $O/icm.json 2>>$O/err.log || exit 1
grep -o '"ms_per_step": [0-9.]*' $O/icm.json | sed "s/^/icm /" >> $O/ab.txt
timeout -k 10 400 python bench.py --steps 2 --warmup 1 > $O/bench.json 2>>$O/err.log || exit 1
grep -o '"ms_per_step": [0-9.]*' $O/bench.json | sed "s/^/full /" >> $O/ab.txt
echo done
