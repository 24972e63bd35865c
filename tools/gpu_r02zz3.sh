# 64-row waves for the conv2 / conv3 split forwards and the conv3 dgrad only (fc / head GEMMs keep
# 32): whole-iteration A/B (same box, alternating) at the 1-GPU shape and the 8-GPU per-rank shape.
set -o pipefail
O=gpurun_out/r02zz3; mkdir -p $O
export TMPDIR=/tmp
for v in mt2all mt2b; do
  PPOX_LIB=$PWD/tools/variants/$v/libppox.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "sg2_conv_big_batch or conv3_wgrad_split_big or split_conv or nature_conv_fwd or trunk_backward" > $O/t_$v.log 2>&1 || { echo FAIL $v; grep -E "^FAILED|Error|assert" $O/t_$v.log | head; tail -3 $O/t_$v.log; exit 1; }
  tail -1 $O/t_$v.log
done
for r in 1 2; do
  for v in main mt2b mt2all; do
    lib=""; [ $v != main ] && lib=$PWD/tools/variants/$v/libppox.so
    PPOX_LIB=$lib timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/b_${v}_$r.json 2>>$O/err.log || exit 1
    echo "$v $r $(grep -o '"ms_per_step": [0-9.]*' $O/b_${v}_$r.json)" | tee -a $O/ab.txt
  done
  for v in main mt2all; do
    lib=""; [ $v != main ] && lib=$PWD/tools/variants/$v/libppox.so
    PPOX_LIB=$lib timeout -k 10 300 python bench.py --envs 512 --batch-size 2048 --steps 3 --warmup 1 --no-cpu-baseline > $O/r_${v}_$r.json 2>>$O/err.log || exit 1
    echo "rank $v $r $(grep -o '"ms_per_step": [0-9.]*' $O/r_${v}_$r.json)" | tee -a $O/ab.txt
  done
done
echo done
