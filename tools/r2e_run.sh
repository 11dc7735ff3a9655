#!/bin/bash
# r2e: GPU tests at HEAD, K1 v1 vs v3 probe, default bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r2e
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/gpu_tests.log 2>&1 || exit $?
tail -3 $OUT/gpu_tests.log
timeout -k 10 400 python -u tools/k1_probe.py --gb 4 --reps 3 --variants 1:0:4096,3:0:2048,3:16:2048,3:144:2048,3:208:2048,3:272:2048,3:464:2048,3:464:4096 > $OUT/k1_probe.log 2>&1 || exit $?
cat $OUT/k1_probe.log
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.log || exit $?
cat $OUT/bench.json
