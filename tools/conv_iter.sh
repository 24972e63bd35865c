#!/bin/bash
# Conv kernel iteration on the GPU box: numerics tests, then per-kernel timing.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "nature or split" > gpurun_out/t_conv.log 2>&1 || { tail -30 gpurun_out/t_conv.log; exit 1; }
tail -2 gpurun_out/t_conv.log
timeout -k 10 200 python tools/conv_bench.py "$@" > gpurun_out/conv_bench.jsonl 2>&1
cat gpurun_out/conv_bench.jsonl | grep -v amdgpu.ids
