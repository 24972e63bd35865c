#!/bin/bash
# Round-end measurement recipe (run via gpurun from the repo root): the default bench line (with the
# cpu_baseline leg), the 8-GPU per-rank shape and the PPO_ICM per-rank shape on one GPU, then the
# rocprof stats / PMC refresh of tools/gpu_profile.sh.  Writes gpurun_out/TAG/.
# Usage: tools/gpu_final.sh TAG
set -o pipefail
TAG=${1:-r03}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 python -u bench.py --envs 512 --batch-size 2048 --steps 5 --warmup 2 --no-cpu-baseline \
    > $O/bench_rank_shape.json 2>> $O/bench.err || exit $?
timeout -k 10 300 python -u bench.py --algo icm --envs 512 --batch-size 2048 --steps 3 --warmup 1 --no-cpu-baseline \
    > $O/bench_icm.json 2>> $O/bench.err || exit $?
tools/gpu_profile.sh $TAG
