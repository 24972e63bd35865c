set -o pipefail
mkdir -p gpurun_out/r02e
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "nature or split or fc or trunk or cnn or conv" > gpurun_out/r02e/tests.log 2>&1 || { echo TESTFAIL; exit 1; }
timeout -k 10 200 python tools/conv_bench.py 16384 > gpurun_out/r02e/conv_new.jsonl 2>&1 || exit 1
timeout -k 10 200 python tools/conv_bench.py 16384 tools/variants/sg0/libppox.so > gpurun_out/r02e/conv_old.jsonl 2>&1 || exit 1
timeout -k 10 200 python tools/fc_bench.py 16384 > gpurun_out/r02e/fc_new.jsonl 2>&1 || exit 1
timeout -k 10 200 python tools/fc_bench.py 16384 tools/variants/sg0/libppox.so > gpurun_out/r02e/fc_old.jsonl 2>&1 || exit 1
timeout -k 10 200 python tools/conv_bench.py 2048 > gpurun_out/r02e/conv_new_2048.jsonl 2>&1 || exit 1
timeout -k 10 200 python tools/conv_bench.py 2048 tools/variants/sg0/libppox.so > gpurun_out/r02e/conv_old_2048.jsonl 2>&1 || exit 1
echo done
