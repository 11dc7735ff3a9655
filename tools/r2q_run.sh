#!/bin/bash
# r2q: K1 v3 guided schedule (lane ranges of 4/2/1 x 1 KiB chunks, '\n' counts as uint16): full GPU tests, probe, bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2q
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/gpu_tests.log 2>&1 || exit $?
tail -3 $OUT/gpu_tests.log
timeout -k 10 300 python -u tools/k1_probe.py --gb 4 --reps 3 --variants 3:464,3:464:2048,3:464:512 > $OUT/probe4g.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/k1_probe.py --gb 1.4 --reps 3 --variants 3:464,3:464:2048 > $OUT/probe1g.log 2>&1 || exit $?
grep -v amdgpu.ids $OUT/probe4g.log $OUT/probe1g.log
timeout -k 10 500 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.log || exit $?
cat $OUT/bench.log
