#!/bin/bash
# r3c (round-2 final state): full GPU tests, smoke, default bench (config 2), config 1, rocprof kernel trace,
# FETCH/WRITE traffic of the bench layout, K1/K2 PMC on a 4 GB resident launch.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3c
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/gpu_tests.log 2>&1 || exit $?
tail -2 $OUT/gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.log || exit $?
cat $OUT/bench.log
timeout -k 10 300 python -u bench.py --config 1 > $OUT/bench_c1.json 2> $OUT/bench_c1.log || exit $?
cat $OUT/bench_c1.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench -- python3 bench.py --no-cpu-baseline --no-resident --steps 3 > $OUT/bench_prof.json 2> $OUT/bench_prof.log || exit $?
bash tools/pmc_traffic.sh $OUT/traffic --steps 1 --warmup 0 --no-resident || exit $?
bash tools/pmc_probe.sh $OUT/pmc --gb 4 --reps 2 || exit $?
