#!/bin/bash
# One GPU session (run via gpurun from the repo root): the named steps in order, each under its own
# time limit; the first failure ends the script (no step runs after a failed GPU step).  Replaces the
# per-session scripts of rounds 2-4 (tools/gpu_r04_*.sh etc.: `git show 66b2eab:tools/...`).
#   tools/gpu.sh TAG STEP [STEP ...]
# Steps (output under gpurun_out/TAG/):
#   tests            the whole GPU suite (PPOX_PARITY_OUT=parity/), tests.log
#   tests:FILES[:K]  pytest on FILES (comma-separated, under tests/) [-k K, "+" for spaces]; =VAR=val,... as below
#   F R RD I ID C3 ES  bench lines: F = the 1-GPU line (20 steps, no cpu baseline), FC = the default line with
#                    the cpu baseline, R = the 8-GPU per-rank shape (512 envs, minibatch 2,048), RD = R with the
#                    data-parallel branches over a one-rank RCCL communicator, I / ID = PPO_ICM per-rank
#                    (+ dp branches), C3 = PPO_RND 1024 x 128, ES = ES-NSRA P = 10,000.  A suffix =VAR=val,...
#                    sets environment variables (e.g. R=PPOX_DCONV2=0); each line -> NAME[_n].json
#   prof16k          rocprofv3 --kernel-trace --stats of the 1-GPU bench + one 16,384-row minibatch timeline
#   profrank[D]      the same at the per-rank shape (D: dp branches forced on) + one 2,048-row minibatch timeline
#   pmc16k / pmcrank FETCH_SIZE / WRITE_SIZE passes (2*FETCH + WRITE per launch) -> pmc_summary{,_rank}.json
#   sq16k / sqrank   SQ counter passes of the MFMA kernels (tools/kernel_pmc.sh)
#   hostlag[D]       tools/host_lag.py at the per-rank shape (PPO; D: dp branches on)
#   hostlagI[D]      the same for PPO_ICM
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
KRX="wgrad|gae|gemm|split_kernel|colp_kernel|planes|dconv|fcd_kernel|dgrad2|ddgrad3|fcw_kernel|fcwg_kernel|hbw_kernel"
SQRX="sgemm|wgrad|colp|fwd1|dconv|fcd_kernel|dgrad2|ddgrad3|fcw_kernel|fcwg_kernel|hbw_kernel"
RANK="--envs 512 --batch-size 2048"

bench() {  # bench NAME OUTFILE ARGS...   (the step's VAR=value settings from $ENVS)
  local name=$1 out=$2; shift 2
  env $ENVS timeout -k 10 400 python3 -u $R/bench.py "$@" > $O/$out.json 2>> $O/bench.err \
      || { echo "bench $name failed" >&2; return 1; }
  cat $O/$out.json
}

trace() {  # trace NAME BACK ARGS... -> stats + timeline of the BACK-th minibatch from the end
  local name=$1 back=$2; shift 2
  ( cd /tmp && env $ENVS timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/$TAG-$name -o run --output-format csv -- \
      python3 $R/bench.py "$@" > $O/${name}_bench_under_rocprof.json 2> $O/$name.err ) || return 1
  local T=$(find /tmp/$TAG-$name -name "*kernel_trace.csv" | head -n 1)
  find /tmp/$TAG-$name -name "*kernel_stats.csv" -exec cp {} $O/${name}_kernel_stats.csv \; || return 1
  python3 $R/tools/trace_by_grid.py $T $O/${name}_kernel_by_grid.csv || return 1
  python3 $R/tools/timeline.py $T $back > $O/${name}_timeline.txt || return 1
}

pmc() {  # pmc NAME ARGS...
  local name=$1; shift
  for C in FETCH_SIZE WRITE_SIZE; do
    ( cd /tmp && timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "$KRX" -d /tmp/$TAG-$name-$C -o run \
        --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --epochs 1 --no-cpu-baseline "$@" \
        > $O/${name}_$C.log 2>&1 ) || return 1
    find /tmp/$TAG-$name-$C -name "*counter_collection.csv" -exec cp {} $O/${name}_$C.csv \; || return 1
  done
  python3 $R/tools/pmc_summary.py $O/${name}_FETCH_SIZE.csv $O/${name}_WRITE_SIZE.csv $O/${name}_summary.json \
      > $O/${name}_summary.txt || return 1
  rm -f $O/${name}_FETCH_SIZE.csv $O/${name}_WRITE_SIZE.csv
}

for STEP in "$@"; do
  echo "[gpu.sh] $STEP $(date +%T)" >&2
  NAME=${STEP%%=*}
  ENVS=""
  [ "$NAME" != "$STEP" ] && ENVS="PPOX_AB=1 $(echo ${STEP#*=} | tr ',' ' ')"
  OUT=$NAME
  [ -n "$ENVS" ] && OUT=${NAME}_$(echo $ENVS | tr ' =' '__' | tr -cd 'A-Za-z0-9_')
  case $NAME in
    tests)
      mkdir -p $O/parity
      PPOX_PARITY_OUT=$O/parity timeout -k 10 1100 python3 -u -m pytest $R/tests -m gpu -x -v --timeout 400 \
          --timeout-method thread > $O/tests.log 2>&1 || exit $?
      tail -n 3 $O/tests.log ;;
    tests:*)
      SPEC=${NAME#tests:}; FILES=${SPEC%%:*}; K=""
      [ "$FILES" != "$SPEC" ] && K=$(echo ${SPEC#*:} | tr "+" " ")
      ARGS=""; for f in $(echo $FILES | tr ',' ' '); do ARGS="$ARGS $R/tests/$f"; done
      [ -n "$ENVS" ] && echo "[gpu.sh] env $ENVS" >> $O/tests_sel.log
      env $ENVS timeout -k 10 900 python3 -u -m pytest $ARGS -x -v --timeout 300 --timeout-method thread ${K:+-k "$K"} \
          >> $O/tests_sel.log 2>&1 || { tail -n 30 $O/tests_sel.log; exit 1; }
      tail -n 3 $O/tests_sel.log ;;
    tsoft:*)
      # tsoft:FILES[:K] — as tests:, but a test failure (pytest rc 1) goes on to the next step (repeat runs of a
      # sporadic failure); a crash / time limit (any other rc) ends the script
      SPEC=${NAME#tsoft:}; FILES=${SPEC%%:*}; K=""
      [ "$FILES" != "$SPEC" ] && K=$(echo ${SPEC#*:} | tr "+" " ")
      ARGS=""; for f in $(echo $FILES | tr ',' ' '); do ARGS="$ARGS $R/tests/$f"; done
      echo "[gpu.sh] tsoft env $ENVS" >> $O/tests_sel.log
      env $ENVS timeout -k 10 600 python3 -u -m pytest $ARGS -x -v --timeout 300 --timeout-method thread ${K:+-k "$K"} \
          >> $O/tests_sel.log 2>&1
      rc=$?
      [ $rc -eq 0 ] || [ $rc -eq 1 ] || { tail -n 30 $O/tests_sel.log; exit $rc; }
      tail -n 1 $O/tests_sel.log ;;
    cstress)
      # the one-process per-rank stress test (tests/test_rank_shape_finite_gpu.py, two streams) while 7 other
      # processes load the same GPU (per-rank bench lines): does a rank pass corrupt under another process's load?
      PIDS=""
      for i in 1 2 3 4 5 6 7; do
        timeout -k 10 300 python3 -u $R/bench.py $RANK --steps 400 --warmup 1 --no-cpu-baseline \
            > $O/cstress_bg$i.json 2> $O/cstress_bg$i.err &
        PIDS="$PIDS $!"
      done
      sleep 60
      env PPOX_STRESS_EPOCHS=120 $ENVS timeout -k 10 400 python3 -u -m pytest $R/tests/test_rank_shape_finite_gpu.py -x -v --timeout 380 \
          --timeout-method thread >> $O/tests_sel.log 2>&1
      rc=$?
      kill $PIDS 2>/dev/null; wait $PIDS 2>/dev/null
      [ $rc -eq 0 ] || [ $rc -eq 1 ] || { tail -n 30 $O/tests_sel.log; exit $rc; }
      tail -n 1 $O/tests_sel.log ;;
    xfail:*)
      # xfail:VARIANT:FILE[:K] — FILE's tests against tools/variants/VARIANT/libppox.so, which must FAIL (pytest
      # rc 1); a crash / time limit (any other rc) ends the script as a failure
      SPEC=${STEP#xfail:}; V=${SPEC%%:*}; REST=${SPEC#*:}; FILE=${REST%%:*}; K=""
      [ "$FILE" != "$REST" ] && K=$(echo ${REST#*:} | tr "+" " ")
      PPOX_LIB=$R/tools/variants/$V/libppox.so timeout -k 10 600 python3 -u -m pytest $R/tests/$FILE -x -v --timeout 300 \
          --timeout-method thread ${K:+-k "$K"} > $O/xfail_$V.log 2>&1
      rc=$?
      tail -n 5 $O/xfail_$V.log
      [ $rc -eq 1 ] || { echo "xfail $V: pytest rc $rc (expected 1)" >&2; exit 1; } ;;
    fcwg) timeout -k 10 300 python3 -u $R/tools/fcwg_bench.py 2048 16384 > $O/fcwg_bench.jsonl 2>> $O/bench.err || exit 1
      cat $O/fcwg_bench.jsonl ;;
    F)  bench F $OUT --steps 20 --warmup 2 --no-cpu-baseline || exit 1 ;;
    FC) bench FC $OUT || exit 1 ;;
    R)  bench R $OUT $RANK --steps 5 --warmup 2 --no-cpu-baseline || exit 1 ;;
    RD) bench RD $OUT $RANK --steps 5 --warmup 2 --no-cpu-baseline --force-dist || exit 1 ;;
    I)  bench I $OUT --algo icm $RANK --steps 3 --warmup 1 --no-cpu-baseline || exit 1 ;;
    ID) bench ID $OUT --algo icm $RANK --steps 3 --warmup 1 --no-cpu-baseline --force-dist || exit 1 ;;
    C3) bench C3 $OUT --algo rnd --envs 1024 --steps 3 --warmup 1 --no-cpu-baseline || exit 1 ;;
    ES) bench ES $OUT --algo es --steps 3 --warmup 1 || exit 1 ;;
    prof16k) trace $OUT 3 --steps 2 --warmup 1 --no-cpu-baseline || exit 1 ;;
    profrank) trace $OUT 3 $RANK --steps 2 --warmup 1 --no-cpu-baseline || exit 1 ;;
    profrankD) trace $OUT 3 $RANK --steps 2 --warmup 1 --no-cpu-baseline --force-dist || exit 1 ;;
    pmc16k) pmc pmc16k || exit 1 ;;
    pmcrank) pmc pmcrank $RANK || exit 1 ;;
    sq16k) $R/tools/kernel_pmc.sh $TAG/sq16k "$SQRX" bench.py --steps 1 --warmup 0 --epochs 1 --no-cpu-baseline || exit 1 ;;
    sqrank) $R/tools/kernel_pmc.sh $TAG/sqrank "$SQRX" bench.py $RANK --steps 1 --warmup 0 --epochs 1 --no-cpu-baseline || exit 1 ;;
    hostlag) timeout -k 10 300 python3 -u $R/tools/host_lag.py 512 2048 ppo x > $O/hostlag.txt 2>> $O/bench.err || exit 1 ;;
    hostlagD) timeout -k 10 300 python3 -u $R/tools/host_lag.py 512 2048 ppo dist > $O/hostlagD.txt 2>> $O/bench.err || exit 1 ;;
    hostlagI) timeout -k 10 300 python3 -u $R/tools/host_lag.py 512 2048 icm x > $O/hostlagI.txt 2>> $O/bench.err || exit 1 ;;
    hostlagID) timeout -k 10 300 python3 -u $R/tools/host_lag.py 512 2048 icm dist > $O/hostlagID.txt 2>> $O/bench.err || exit 1 ;;
    *) echo "unknown step $STEP" >&2; exit 2 ;;
  esac
done
echo done > $O/DONE
