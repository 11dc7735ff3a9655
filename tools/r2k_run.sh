#!/bin/bash
# r2k: re-run of HEAD after the container reset (r2d-r2j outputs were lost): GPU tests, probe, bench, rocprof.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2k
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/gpu_tests.log 2>&1 || exit $?
tail -3 $OUT/gpu_tests.log
timeout -k 10 300 python -u tools/k1_probe.py --gb 4 --reps 4 > $OUT/k1_probe_4g.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/k1_probe.py --gb 1 --reps 4 > $OUT/k1_probe_1g.log 2>&1 || exit $?
cat $OUT/k1_probe_4g.log $OUT/k1_probe_1g.log
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.log || exit $?
cat $OUT/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench -- python3 bench.py --no-cpu-baseline --no-resident --steps 3 > $OUT/bench_prof.json 2> $OUT/bench_prof.log || exit $?
