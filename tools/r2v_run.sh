#!/bin/bash
# r2v: guided K1 schedule (1 KiB / 2 KiB chunks, one round each of 2- and 1-chunk ranges), K2 one hit per thread:
# full GPU tests, smoke, bench, rocprof kernel trace, FETCH/WRITE traffic of the bench layout, K1 PMC.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2v
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/gpu_tests.log 2>&1 || exit $?
tail -2 $OUT/gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.log || exit $?
cat $OUT/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench -- python3 bench.py --no-cpu-baseline --no-resident --steps 3 > $OUT/bench_prof.json 2> $OUT/bench_prof.log || exit $?
bash tools/pmc_traffic.sh $OUT/traffic --steps 1 --warmup 0 --no-resident || exit $?
bash tools/pmc_probe.sh $OUT/pmc --gb 4 --reps 2 || exit $?
