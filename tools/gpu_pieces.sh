#!/bin/bash
# Pipeline split sweep of the default bench (pieces:first-piece share).
#   tools/gpu_pieces.sh TAG [P:F ...]
set -o pipefail
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for PF in ${@:-1:0.5 2:0.6 2:0.7}; do
  P=${PF%%:*}; F=${PF##*:}
  TSG_PIECES=$P TSG_FIRST_PIECE=$F timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --json-out $OUT/bench_p${P}_$F.json > /dev/null 2> $OUT/bench_p${P}_$F.log || exit $?
  echo "pieces=$P first=$F"; grep step $OUT/bench_p${P}_$F.log
done
