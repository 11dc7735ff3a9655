#!/bin/bash
# r3k: three-pass CR strip with batched scan loads: parity tests, timing at three densities, rocprof split.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3k
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_cr_strip.py > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
OUT=$OUT bash tools/r3e_run.sh
