# graph-captured collect: test, full suite, bench lines
set -o pipefail
O=gpurun_out/r02y; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_product_gpu.py -m gpu -x -q -k "collect_graph" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/t0.log 2>&1 || { echo FAIL0; tail -30 $O/t0.log; exit 1; }
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { echo FAIL; grep -E "^FAILED|Error" $O/t.log | head -20; tail -3 $O/t.log; exit 1; }
timeout -k 10 300 python bench.py --envs 512 --batch-size 2048 --steps 3 --warmup 1 --no-cpu-baseline > $O/rank.json 2>$O/rank.err || exit 1
PPOX_COLLECT_GRAPH=0 timeout -k 10 300 python bench.py --envs 512 --batch-size 2048 --steps 3 --warmup 1 --no-cpu-baseline > $O/rank_nograph.json 2>$O/rank_ng.err || exit 1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench.json 2>$O/bench.err || exit 1
echo done
