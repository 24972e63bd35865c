# A/B conv + fc timing of variant builds: tools/gpu_ab3.sh TAG B variant...   ("main" = in-tree lib)
set -o pipefail
TAG=$1; B=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
for r in 1 2; do
  for v in "$@"; do
    lib=""; [ $v != main ] && lib=$PWD/tools/variants/$v/libppox.so
    timeout -k 10 200 python tools/conv_bench.py $B $lib > $O/c_${v}_$r.jsonl 2>&1 || exit 1
    timeout -k 10 200 python tools/fc_bench.py $B $lib > $O/f_${v}_$r.json 2>&1 || exit 1
  done
done
echo done
