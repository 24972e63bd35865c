set -o pipefail
mkdir -p gpurun_out/r02k
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r02k/tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r02k/tests.log; exit 1; }
for v in main g8 g4 g1; do
  lib=""; [ $v != main ] && lib=tools/variants/$v/libppox.so
  timeout -k 10 200 python tools/fc_bench.py 16384 $lib > gpurun_out/r02k/fc_$v.jsonl 2>&1 || exit 1
done
timeout -k 10 200 python tools/conv_bench.py 16384 > gpurun_out/r02k/conv_main.jsonl 2>&1 || exit 1
echo done
