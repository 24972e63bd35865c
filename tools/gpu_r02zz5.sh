# Backward stream schedule A/B after the split-f16 change (env switches only): two streams (default),
# one stream, and the conv2 dgrad beside wgrad2 at every batch.
set -o pipefail
O=gpurun_out/r02zz5; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for v in default one nosolo; do
    case $v in default) E="";; one) E="PPOX_BWD_STREAMS=0";; nosolo) E="PPOX_BWD_SOLO_DGRAD2=1000000";; esac
    env $E timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/b_${v}_$r.json 2>>$O/err.log || exit 1
    echo "$v $r $(grep -o '"ms_per_step": [0-9.]*' $O/b_${v}_$r.json)" | tee -a $O/ab.txt
  done
done
echo done
