#!/bin/bash
# Round-4 full check (run via gpurun): the whole GPU suite with the parity reports
# (PPOX_PARITY_OUT -> gpurun_out/TAG/parity/*.json), the bench line (+ cpu_baseline), the per-rank
# shapes: PPO, PPO_ICM, and PPO_ICM with the data-parallel paths forced on over a one-rank RCCL
# communicator (the 8-GPU per-rank program).  Writes gpurun_out/TAG/.
set -o pipefail
TAG=${1:-r04full}
O=gpurun_out/$TAG
mkdir -p $O/parity
PPOX_PARITY_OUT=$O/parity timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 \
    --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 python -u bench.py --envs 512 --batch-size 2048 --steps 5 --warmup 2 --no-cpu-baseline \
    > $O/bench_rank_shape.json 2>> $O/bench.err || exit $?
timeout -k 10 300 python -u bench.py --algo icm --envs 512 --batch-size 2048 --steps 3 --warmup 1 --no-cpu-baseline \
    > $O/bench_icm.json 2>> $O/bench.err || exit $?
timeout -k 10 300 python -u bench.py --algo icm --envs 512 --batch-size 2048 --steps 3 --warmup 1 --no-cpu-baseline \
    --force-dist > $O/bench_icm_dist.json 2>> $O/bench.err || exit $?
timeout -k 10 300 python -u bench.py --envs 512 --batch-size 2048 --steps 5 --warmup 2 --no-cpu-baseline \
    --force-dist > $O/bench_rank_shape_dist.json 2>> $O/bench.err || exit $?
for B in 2048 16384; do
  timeout -k 10 200 python -u tools/graph_probe.py $B 40 > $O/graph_probe_$B.log 2>&1 || exit $?
done
echo done > $O/DONE
