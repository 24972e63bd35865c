# sg2 with 64 rows per wave (SG_MT=2 variant): bitwise + time vs in-tree for fwd2 / fwd3 / dgrad3
# and the fc GEMMs, then whole-iteration A/B (same box, alternating).
set -o pipefail
O=gpurun_out/r02zz2; mkdir -p $O
export TMPDIR=/tmp
V=$PWD/tools/variants/mt2/libppox.so
for B in 16384 2048 2311; do
  timeout -k 10 200 python tools/split_ab.py $B $V >> $O/split_ab.jsonl 2>>$O/err.log || exit 1
done
cat $O/split_ab.jsonl
timeout -k 10 200 python tools/fc_bench.py 16384 > $O/fc_main.jsonl 2>>$O/err.log || exit 1
timeout -k 10 200 python tools/fc_bench.py 16384 $V > $O/fc_mt2.jsonl 2>>$O/err.log || exit 1
for r in 1 2; do
  for v in main mt2; do
    lib=""; [ $v != main ] && lib=$V
    PPOX_LIB=$lib timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/b_${v}_$r.json 2>>$O/err.log || exit 1
    echo "$v $r $(grep -o '"ms_per_step": [0-9.]*' $O/b_${v}_$r.json)" | tee -a $O/ab.txt
  done
done
echo done
