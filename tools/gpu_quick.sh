#!/bin/bash
# GPU tests + default bench (no CPU baseline) + config 3 bench.
#   tools/gpu_quick.sh TAG
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit $?
tail -2 $OUT/gpu_tests.log
timeout -k 10 200 python bench.py --no-cpu-baseline --no-pcie --steps 5 --json-out $OUT/bench.json > /dev/null 2> $OUT/bench.log || exit $?
grep step $OUT/bench.log
timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline --no-pcie --steps 3 --json-out $OUT/bench_c3.json > /dev/null 2> $OUT/bench_c3.log || exit $?
grep step $OUT/bench_c3.log
