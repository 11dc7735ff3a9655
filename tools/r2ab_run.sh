#!/bin/bash
# A/B of two in-tree builds on one box (TSG_LIB): config 3 bench, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2ab
mkdir -p $OUT
for i in 1 2; do
  for v in libtrivysecret_a.so libtrivysecret.so; do
    TSG_LIB=$v timeout -k 10 300 python -u bench.py --config 3 --no-cpu-baseline --steps 2 --warmup 1 --gb 5 > $OUT/c3_${v}_$i.json 2> $OUT/c3_${v}_$i.log || exit $?
    echo "$v $i: $(grep -h 'step\|HBM' $OUT/c3_${v}_$i.log | cut -c1-160 | tr '\n' ' ')"
  done
done
