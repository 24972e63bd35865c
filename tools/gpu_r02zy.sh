# A/B of compile-time knobs (wgrad KT per layer, pixels per split, sg2 ring slots): conv_bench
# of the in-tree libppox vs each variant, at the 1-GPU minibatch and the 8-GPU per-rank one.
set -o pipefail
O=gpurun_out/r02zy; mkdir -p $O
export TMPDIR=/tmp
for B in 16384 2048; do
  timeout -k 10 200 python tools/conv_bench.py $B > $O/base_$B.jsonl 2>>$O/err.log || exit 1
  for v in kt2_256 kt3_192 px1024 slots3; do
    timeout -k 10 200 python tools/conv_bench.py $B tools/variants/$v/libppox.so > $O/${v}_$B.jsonl 2>>$O/err.log || exit 1
  done
done
echo done
