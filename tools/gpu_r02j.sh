set -o pipefail
mkdir -p gpurun_out/r02j
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "nature or split or fc or trunk or cnn or conv" > gpurun_out/r02j/tests.log 2>&1 || { echo TESTFAIL; exit 1; }
for v in main sg8 sg0; do
  lib=""; [ $v != main ] && lib=tools/variants/$v/libppox.so
  timeout -k 10 200 python tools/conv_bench.py 16384 $lib > gpurun_out/r02j/conv_$v.jsonl 2>&1 || exit 1
  timeout -k 10 200 python tools/fc_bench.py 16384 $lib > gpurun_out/r02j/fc_$v.jsonl 2>&1 || exit 1
  timeout -k 10 200 python tools/conv_bench.py 2048 $lib > gpurun_out/r02j/conv2048_$v.jsonl 2>&1 || exit 1
  timeout -k 10 200 python tools/fc_bench.py 2048 $lib > gpurun_out/r02j/fc2048_$v.jsonl 2>&1 || exit 1
done
echo done
