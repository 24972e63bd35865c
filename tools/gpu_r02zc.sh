set -o pipefail
O=gpurun_out/r02zc; mkdir -p $O
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 400 python -u -m pytest tests/test_icm_gpu.py -v -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/t_icm.log 2>&1 || { echo FAIL; grep -E "^FAILED|Error|assert" $O/t_icm.log | head -30; tail -3 $O/t_icm.log; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py tests/test_configs_gpu.py tests/test_product_gpu.py -q -x -k "ICM or icm" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/t_icm2.log 2>&1 || { echo FAIL2; grep -E "^FAILED|Error|assert" $O/t_icm2.log | head -30; tail -3 $O/t_icm2.log; exit 1; }
timeout -k 10 300 python bench.py --algo icm --envs 512 --batch-size 2048 --steps 2 --warmup 1 --no-cpu-baseline > $O/icm.json 2>$O/icm.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/rz -o run --output-format csv -- \
    python3 $R/bench.py --algo icm --envs 512 --batch-size 2048 --steps 1 --warmup 1 --no-cpu-baseline > $O/icm_prof.log 2>&1 || exit 1
cp /tmp/rz/*kernel_stats* $O/icm_kernel_stats.csv
echo done
