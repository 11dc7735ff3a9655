#!/bin/bash
# r2f: GPU tests (K1 v3/464 default, host keyword gate fix), v3 ablations, bench, rocprof of bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2f
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/gpu_tests.log 2>&1 || exit $?
tail -3 $OUT/gpu_tests.log
timeout -k 10 400 python -u tools/k1_probe.py --gb 4 --reps 3 --variants 1:0:4096,3:464:4096,3:400:4096,3:448:4096,3:464:8192,3:465:4096,3:466:4096,3:468:4096,3:472:4096,3:496:4096 > $OUT/k1_probe.log 2>&1 || exit $?
cat $OUT/k1_probe.log
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.log || exit $?
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench -- python3 bench.py --no-cpu-baseline --steps 3 > $OUT/bench_prof.json 2> $OUT/bench_prof.log || exit $?
find $OUT/prof -name "*stats*"
