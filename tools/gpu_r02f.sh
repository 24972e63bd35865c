set -o pipefail
mkdir -p gpurun_out/r02f
for v in main nodma nosplit; do
  lib=""; [ $v != main ] && lib=tools/variants/$v/libppox.so
  timeout -k 10 200 python tools/conv_bench.py 16384 $lib > gpurun_out/r02f/conv_$v.jsonl 2>&1 || exit 1
  timeout -k 10 200 python tools/fc_bench.py 16384 $lib > gpurun_out/r02f/fc_$v.jsonl 2>&1 || exit 1
done
echo done
