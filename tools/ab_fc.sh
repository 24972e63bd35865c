# same-box A/B of the fc-layer forms (dev tool)
for v in 1 0; do
  PPOX_FC_DGRAD_FUSED_MAX=$([ $v = 1 ] && echo 1000000 || echo 0) timeout -k 10 300 python bench.py --no-cpu-baseline 2>&1 | grep -o '"ms_per_step": [0-9.]*' | sed "s/^/full fused=$v /"
  PPOX_FC_DGRAD_FUSED_MAX=$([ $v = 1 ] && echo 1000000 || echo 0) timeout -k 10 300 python bench.py --no-cpu-baseline --envs 512 --batch-size 2048 --steps 5 2>&1 | grep -o '"ms_per_step": [0-9.]*' | sed "s/^/small fused=$v /"
done
