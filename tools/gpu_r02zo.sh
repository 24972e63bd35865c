set -o pipefail
O=gpurun_out/r02zo; mkdir -p $O
for v in main pb16 pb4 main; do
  lib=""; [ $v != main ] && lib=$PWD/tools/variants/$v/libppox.so
  PPOX_LIB=$lib timeout -k 10 200 python tools/icm_bench.py 2048 | sed "s/^/$v /" >> $O/icm.txt 2>>$O/err.log || exit 1
done
timeout -k 10 200 python tools/icm_bench.py 512 | sed "s/^/main512 /" >> $O/icm.txt 2>>$O/err.log || exit 1
echo done
