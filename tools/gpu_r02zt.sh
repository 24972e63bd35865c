set -o pipefail
O=gpurun_out/r02zt; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gae_gpu.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { echo FAIL; grep -E "^FAILED|Error" $O/t.log | head; tail -3 $O/t.log; exit 1; }
timeout -k 10 300 python tools/gae_sweep.py > $O/gae_sweep.jsonl 2>>$O/err.log || exit 1
echo done
