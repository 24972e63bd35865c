set -o pipefail
O=gpurun_out/r02zi; mkdir -p $O
for B in 512 1000 2048 4096 8192; do
  timeout -k 10 200 python tools/fc_bench.py $B >> $O/fc.jsonl 2>>$O/err.log || exit 1
done
echo done
