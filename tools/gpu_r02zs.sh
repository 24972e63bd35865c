set -o pipefail
O=gpurun_out/r02zs; mkdir -p $O
for v in main cu32 cu64 main cu32 cu64; do
  lib=""; [ $v != main ] && lib=$PWD/tools/variants/$v/libppox.so
  PPOX_LIB=$lib timeout -k 10 300 python bench.py --envs 512 --batch-size 2048 --steps 3 --warmup 1 --no-cpu-baseline > $O/rank_$v.json 2>>$O/err.log || exit 1
  grep -o '"ms_per_step": [0-9.]*' $O/rank_$v.json | sed "s/^/rank $v /" >> $O/ab.txt
done
for v in main cu32; do
  lib=""; [ $v != main ] && lib=$PWD/tools/variants/$v/libppox.so
  PPOX_LIB=$lib timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/full_$v.json 2>>$O/err.log || exit 1
  grep -o '"ms_per_step": [0-9.]*' $O/full_$v.json | sed "s/^/full $v /" >> $O/ab.txt
done
echo done
