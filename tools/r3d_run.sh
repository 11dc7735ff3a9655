#!/bin/bash
# r3d: GPU CR strip parity tests, then the default bench (config 2) with the CR strip leg.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3d
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_cr_strip.py > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 500 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.log || { tail -30 $OUT/bench.log; exit 1; }
cat $OUT/bench.log
