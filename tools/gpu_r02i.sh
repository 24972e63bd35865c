set -o pipefail
mkdir -p gpurun_out/r02i
for v in nodma p1 p2 p3; do
  timeout -k 10 200 python tools/conv_bench.py 16384 tools/variants/$v/libppox.so > gpurun_out/r02i/conv_$v.jsonl 2>&1 || exit 1
done
echo done
