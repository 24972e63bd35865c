# wgrad tiling variants: correctness (kernel tests on each variant) + conv timing
set -o pipefail
O=gpurun_out/r02m; mkdir -p $O
for v in main w2_256 w3_192; do
  lib=""; [ $v != main ] && lib=$PWD/tools/variants/$v/libppox.so
  PPOX_LIB=$lib timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -k "wgrad or split_conv" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/t_$v.log 2>&1 || { echo FAIL $v; tail -20 $O/t_$v.log; exit 1; }
  timeout -k 10 200 python tools/conv_bench.py 16384 $lib > $O/c_$v.jsonl 2>&1 || exit 1
  timeout -k 10 200 python tools/conv_bench.py 2048 $lib > $O/c2k_$v.jsonl 2>&1 || exit 1
done
echo done
