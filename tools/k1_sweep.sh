#!/bin/bash
# K1 configuration sweep on the GPU box: bench.py (no CPU baseline) once per
# configuration "threads,streams,chunk" (TSG_K1_CFG / TSG_K1_CHUNK).
# Usage: tools/k1_sweep.sh OUTDIR cfg1 cfg2 ...
set -o pipefail
OUT=$1; shift
mkdir -p $OUT
for cfg in "$@"; do
  IFS=, read t k c <<< "$cfg"
  tag=${t}_${k}_${c}
  TSG_K1_CFG=$t,$k TSG_K1_CHUNK=$c timeout -k 10 150 python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} \
    > $OUT/bench_$tag.json 2> $OUT/bench_$tag.log || exit $?
  echo "cfg $cfg: $(grep -o '"value": [0-9.]*' $OUT/bench_$tag.json) $(grep '\[bench\] step' $OUT/bench_$tag.log)"
done
