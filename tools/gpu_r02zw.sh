set -o pipefail
O=gpurun_out/r02zw; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_product_gpu.py tests/test_icm_gpu.py tests/test_rccl_gpu.py tests/test_dist_gpu.py tests/test_configs_gpu.py -q -x --timeout 250 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { echo FAIL; grep -E "^FAILED|Error|assert" $O/t.log | head; tail -3 $O/t.log; exit 1; }
for g in 1 0; do
  PPOX_COLLECT_GRAPH=$g timeout -k 10 300 python bench.py --algo icm --envs 512 --batch-size 2048 --steps 2 --warmup 1 --no-cpu-baseline > $O/icm_$g.json 2>>$O/err.log || exit 1
  grep -o '"ms_per_step": [0-9.]*\|"collect": {"gpu_ms": [0-9.]*' $O/icm_$g.json | tr '\n' ' ' | sed "s/^/icm graph=$g /" >> $O/ab.txt; echo >> $O/ab.txt
done
echo done
