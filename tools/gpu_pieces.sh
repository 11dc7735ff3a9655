#!/bin/bash
# GPU tests, then a pipeline-piece sweep of the default bench, then configs 5/3.
#   tools/gpu_pieces.sh TAG
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit $?
tail -2 $OUT/gpu_tests.log
for P in 1 2 4 8; do
  TSG_PIECES=$P timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --json-out $OUT/bench_p$P.json > /dev/null 2> $OUT/bench_p$P.log || exit $?
  echo "pieces=$P"; grep step $OUT/bench_p$P.log
done
