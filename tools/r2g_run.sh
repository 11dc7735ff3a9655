#!/bin/bash
# r2g: K1 v3 launch-size sweep (1 / 2 / 4 GB x chunk), anchor extension 1, 512-entry wave hit buffers.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r2g
mkdir -p $OUT
for gb in 1 2; do
  timeout -k 10 300 python -u tools/k1_probe.py --gb $gb --reps 4 --variants 3:464:1024,3:464:2048,3:464:4096,3:464:8192 > $OUT/k1_probe_${gb}g.log 2>&1 || exit $?
  cat $OUT/k1_probe_${gb}g.log
done
timeout -k 10 300 python -u tools/k1_probe.py --gb 4 --reps 4 --variants 3:464:2048,3:464:4096 > $OUT/k1_probe_4g.log 2>&1 || exit $?
cat $OUT/k1_probe_4g.log
for gb in 1 4; do
  TSG_ANCHOR_EXT=1 timeout -k 10 300 python -u tools/k1_probe.py --gb $gb --reps 4 --variants 3:464:2048,3:464:4096 > $OUT/k1_probe_ext1_${gb}g.log 2>&1 || exit $?
  cat $OUT/k1_probe_ext1_${gb}g.log
done
