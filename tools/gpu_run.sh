#!/bin/bash
# The one GPU-box runner (replaces the per-run r*_run.sh scripts of rounds 1-2).
#   tools/gpu_run.sh TAG STEP [STEP ...]
# run from the repo root on the box; every step has its own time limit, the
# steps are chained (the first failure ends the call), outputs go to
# gpurun_out/TAG/.  Steps:
#   tests[:PYTEST-ARGS]        pytest -m gpu (default: the whole GPU suite)
#   smoke                      __graft_entry__.smoke()
#   bench[:NAME[:ARGS]]        python bench.py ARGS > NAME.json (NAME default bench)
#   prof[:NAME[:ARGS]]         rocprofv3 --kernel-trace --stats of bench.py ARGS
#   pmc[:NAME[:ARGS]]          tools/pmc_k1.sh passes over bench.py ARGS
#   traffic[:NAME[:ARGS]]      tools/pmc_traffic.sh (FETCH_SIZE / WRITE_SIZE) over bench.py ARGS
#   py:NAME:SECONDS:SCRIPT ARGS   python -u SCRIPT ARGS under its own limit
#   bin:NAME:SECONDS:PROGRAM ARGS a built tool (e.g. tools/load_probe) under its own limit
#   env:NAME=VALUE             export NAME=VALUE for the following steps ("env:NAME=" unsets it)
# e.g. tools/gpu_run.sh rd3a tests smoke bench "bench:c1:--config 1" prof
set -o pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
for STEP in "$@"; do
  KIND=${STEP%%:*}
  REST=${STEP#*:}; [ "$REST" = "$STEP" ] && REST=""
  NAME=${REST%%:*}
  ARGS=${REST#*:}; [ "$ARGS" = "$REST" ] && ARGS=""
  echo "== $STEP" >&2
  case $KIND in
    tests)
      timeout -k 10 1200 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${REST:-tests/} \
        > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
      tail -2 $OUT/gpu_tests.log ;;
    smoke)
      timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
        || { cat $OUT/smoke.log; exit 1; }
      cat $OUT/smoke.log ;;
    bench)
      N=${NAME:-bench}
      timeout -k 10 900 python -u bench.py $ARGS > $OUT/$N.json 2> $OUT/$N.log || { tail -30 $OUT/$N.log; exit 1; }
      grep -E 'step|ceiling|resident|parity|cpu base|launcher' $OUT/$N.log ;;
    prof)
      N=${NAME:-prof}
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/$N -o $N -- \
        python3 $ROOT/bench.py ${ARGS:---no-cpu-baseline --steps 3} > $OUT/$N.json 2> $OUT/$N.log \
        || { tail -20 $OUT/$N.log; exit 1; }
      grep step $OUT/$N.log ;;
    pmc)
      bash tools/pmc_k1.sh $OUT/${NAME:-pmc} $ARGS || exit 1 ;;
    traffic)
      bash tools/pmc_traffic.sh $OUT/${NAME:-traffic} $ARGS || exit 1 ;;
    env)
      if [ -n "${REST#*=}" ]; then export "$REST"; else unset "${REST%%=*}"; fi ;;
    bin)
      SECS=${ARGS%%:*}; CMD=${ARGS#*:}
      timeout -k 10 $SECS $CMD > $OUT/$NAME.log 2>&1 || { tail -30 $OUT/$NAME.log; exit 1; }
      tail -20 $OUT/$NAME.log ;;
    py)
      SECS=${ARGS%%:*}; SCRIPT=${ARGS#*:}
      timeout -k 10 $SECS python -u $SCRIPT > $OUT/$NAME.log 2>&1 || { tail -30 $OUT/$NAME.log; exit 1; }
      tail -15 $OUT/$NAME.log ;;
    *)
      echo "unknown step $STEP" >&2; exit 2 ;;
  esac
done
echo "gpu_run $TAG done"
