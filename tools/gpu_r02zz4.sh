# Weight-gradient grids in whole rounds of the chip's workgroup slots (WS_ROUNDS variant):
# parity tests on the variant, conv kernel times, then whole-iteration A/B at both shapes.
set -o pipefail
O=gpurun_out/r02zz4; mkdir -p $O
export TMPDIR=/tmp
V=$PWD/tools/variants/wsr/libppox.so
PPOX_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_product_gpu.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "wgrad or split_conv or trunk_backward or cnn or atari" > $O/t.log 2>&1 || { echo FAIL; grep -E "^FAILED|Error|assert" $O/t.log | head; tail -3 $O/t.log; exit 1; }
tail -1 $O/t.log
for B in 16384 2048; do
  timeout -k 10 200 python tools/conv_bench.py $B > $O/cb_main_$B.jsonl 2>>$O/err.log || exit 1
  timeout -k 10 200 python tools/conv_bench.py $B $V > $O/cb_wsr_$B.jsonl 2>>$O/err.log || exit 1
done
for r in 1 2; do
  for v in main wsr; do
    lib=""; [ $v != main ] && lib=$V
    PPOX_LIB=$lib timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/b_${v}_$r.json 2>>$O/err.log || exit 1
    echo "$v $r $(grep -o '"ms_per_step": [0-9.]*' $O/b_${v}_$r.json)" | tee -a $O/ab.txt
    PPOX_LIB=$lib timeout -k 10 300 python bench.py --envs 512 --batch-size 2048 --steps 3 --warmup 1 --no-cpu-baseline > $O/r_${v}_$r.json 2>>$O/err.log || exit 1
    echo "rank $v $r $(grep -o '"ms_per_step": [0-9.]*' $O/r_${v}_$r.json)" | tee -a $O/ab.txt
  done
done
echo done
