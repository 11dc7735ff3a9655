#!/bin/bash
# r2y: indexed global AllowPath (config 3's light files): GPU tests, config 3 bench (pinned + resident).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2y
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/gpu_tests.log 2>&1 || exit $?
tail -2 $OUT/gpu_tests.log
timeout -k 10 600 python -u bench.py --config 3 > $OUT/bench_c3.json 2> $OUT/bench_c3.log || exit $?
cat $OUT/bench_c3.log
