# wgrad pipeline: kernel tests + conv timing
set -o pipefail
O=gpurun_out/r02o; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "rollout_rows or wgrad" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/t0.log 2>&1 || { echo FAIL0; tail -30 $O/t0.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { echo FAIL; tail -30 $O/t.log; exit 1; }
timeout -k 10 200 python tools/conv_bench.py 16384 > $O/c.jsonl 2>&1 || exit 1
timeout -k 10 200 python tools/conv_bench.py 2048 > $O/c2k.jsonl 2>&1 || exit 1
echo done
