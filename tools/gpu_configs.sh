#!/bin/bash
# Config-3 / config-5 bench lines on the box (after tools/gpu_full.sh).
#   tools/gpu_configs.sh TAG
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python bench.py --config 5 --gb 2 --steps 2 --cpu-sample-mb 150 --json-out $OUT/bench_c5.json > $OUT/bench_c5.out 2> $OUT/bench_c5.log || exit $?
cat $OUT/bench_c5.log
timeout -k 10 300 python bench.py --config 3 --gb 10 --steps 3 --cpu-sample-mb 600 --json-out $OUT/bench_c3.json > $OUT/bench_c3.out 2> $OUT/bench_c3.log || exit $?
cat $OUT/bench_c3.log
