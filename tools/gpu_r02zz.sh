# conv3 wgrad KT 192 from 8192 rows + the forward ring-slot knob: parity tests, then whole-iteration
# A/B (same box, alternating): main = in-tree, kt3big64 = the previous conv3 wgrad, fwdslots3.
set -o pipefail
O=gpurun_out/r02zz; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "conv3_wgrad or split_conv or nature or split_f16" > $O/t.log 2>&1 || { echo FAIL; grep -E "^FAILED|Error|assert" $O/t.log | head; tail -3 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 1 2; do
  for v in main kt3big64 fwdslots3; do
    lib=""; [ $v != main ] && lib=$PWD/tools/variants/$v/libppox.so
    PPOX_LIB=$lib timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/b_${v}_$r.json 2>>$O/err.log || exit 1
    echo "$v $r $(grep -o '"ms_per_step": [0-9.]*' $O/b_${v}_$r.json)" | tee -a $O/ab.txt
  done
done
timeout -k 10 200 python tools/conv_bench.py 16384 > $O/cb_main.jsonl 2>>$O/err.log || exit 1
timeout -k 10 200 python tools/conv_bench.py 16384 tools/variants/fwdslots3/libppox.so > $O/cb_fwdslots3.jsonl 2>>$O/err.log || exit 1
echo done
