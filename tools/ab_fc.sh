# same-box A/B of the fc-layer forms (dev tool): split-bf16 fc forward from batch MIN
# (PPOX_FC_SPLIT_MIN) and fused split fc dgrad up to batch MAX (PPOX_FC_DGRAD_FUSED_MAX)
for cfg in "1099511627776 8192" "1099511627776 1099511627776" "8192 1099511627776" "1024 1099511627776"; do
  set -- $cfg
  PPOX_FC_SPLIT_MIN=$1 PPOX_FC_DGRAD_FUSED_MAX=$2 timeout -k 10 300 python bench.py --no-cpu-baseline 2>&1 | grep -o '"ms_per_step": [0-9.]*' | sed "s/^/full min=$1 max=$2 /"
  PPOX_FC_SPLIT_MIN=$1 PPOX_FC_DGRAD_FUSED_MAX=$2 timeout -k 10 300 python bench.py --no-cpu-baseline --envs 512 --batch-size 2048 --steps 5 2>&1 | grep -o '"ms_per_step": [0-9.]*' | sed "s/^/small min=$1 max=$2 /"
done
