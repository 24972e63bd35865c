# direct conv3 kernels: kernel tests, then A/B timing vs the im2col sgemm forms
set -o pipefail
O=gpurun_out/r02u; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "split_conv or conv_fwd or dgrad or nature" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/t0.log 2>&1 || { echo FAIL0; tail -30 $O/t0.log; exit 1; }
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { echo FAIL; grep -E "^FAILED|Error" $O/t.log | head -20; tail -3 $O/t.log; exit 1; }
for r in 1 2; do
  for v in main c3old; do
    lib=""; [ $v != main ] && lib=$PWD/tools/variants/$v/libppox.so
    timeout -k 10 200 python tools/conv_bench.py 16384 $lib > $O/c_${v}_$r.jsonl 2>&1 || exit 1
    timeout -k 10 200 python tools/conv_bench.py 2048 $lib > $O/c2k_${v}_$r.jsonl 2>&1 || exit 1
  done
done
echo done
