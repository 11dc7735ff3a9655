#!/bin/bash
# r2h: is K1's fixed per-launch cost clock ramp-up?  1 / 4 GB launches with and without a busy GPU right before.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r2h
mkdir -p $OUT
for pw in 0 5; do
  for gb in 1 4; do
    timeout -k 10 300 python -u tools/k1_probe.py --gb $gb --reps 4 --prewarm-ms $pw --variants 3:464:1024,3:464:4096,3:496:4096 > $OUT/k1_pw${pw}_${gb}g.log 2>&1 || exit $?
    cat $OUT/k1_pw${pw}_${gb}g.log
  done
done
