# full GPU suite on the rebuilt library + ICM / PPO per-rank bench lines
set -o pipefail
O=gpurun_out/r02w; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { echo FAIL; grep -E "^FAILED|Error" $O/t.log | head -20; tail -3 $O/t.log; exit 1; }
timeout -k 10 300 python bench.py --algo icm --envs 512 --batch-size 2048 --steps 2 --warmup 1 --no-cpu-baseline > $O/icm.json 2>$O/icm.err || exit 1
timeout -k 10 300 python bench.py --envs 512 --batch-size 2048 --steps 3 --warmup 1 --no-cpu-baseline > $O/rank.json 2>$O/rank.err || exit 1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench.json 2>$O/bench.err || exit 1
echo done
