set -o pipefail
O=gpurun_out/r02zh; mkdir -p $O
export TMPDIR=/tmp
for s in 1 0 1 0; do
  PPOX_BWD_STREAMS=$s timeout -k 10 300 python bench.py --algo rnd --envs 1024 --batch-size 16384 --steps 2 --warmup 1 --no-cpu-baseline > $O/rnd_$s.json 2>>$O/err.log || exit 1
  grep -o '"ms_per_step": [0-9.]*' $O/rnd_$s.json | sed "s/^/rnd streams=$s /" >> $O/ab.txt
done
for s in 1 0; do
  PPOX_BWD_STREAMS=$s timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/full_$s.json 2>>$O/err.log || exit 1
  grep -o '"ms_per_step": [0-9.]*' $O/full_$s.json | sed "s/^/full streams=$s /" >> $O/ab.txt
done
echo done
