# fc wgrad split kernel: kernel + product tests, fc/conv timing
set -o pipefail
O=gpurun_out/r02q; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "fc_wgrad" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/t0.log 2>&1 || { echo FAIL0; tail -30 $O/t0.log; exit 1; }
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { echo FAIL; grep -E "^FAILED|Error" $O/t.log | head -20; tail -3 $O/t.log; exit 1; }
timeout -k 10 200 python tools/fc_bench.py 16384 > $O/fc16k.jsonl 2>&1 || exit 1
timeout -k 10 200 python tools/fc_bench.py 2048 > $O/fc2k.jsonl 2>&1 || exit 1
echo done
