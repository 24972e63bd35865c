set -o pipefail
O=gpurun_out/r02zm; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { echo FAIL; grep -E "^FAILED|Error" $O/t.log | head -20; tail -3 $O/t.log; exit 1; }
for s in 1 0; do
  PPOX_BWD_STREAMS=$s timeout -k 10 300 python bench.py --algo icm --envs 512 --batch-size 2048 --steps 2 --warmup 1 --no-cpu-baseline > $O/icm_$s.json 2>>$O/err.log || exit 1
  grep -o '"ms_per_step": [0-9.]*\|"collect": {"gpu_ms": [0-9.]*' $O/icm_$s.json | tr '\n' ' ' | sed "s/^/icm streams=$s /" >> $O/ab.txt; echo >> $O/ab.txt
done
echo done
