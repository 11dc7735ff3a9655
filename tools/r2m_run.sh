#!/bin/bash
# r2m: K1 v3 line width / unroll / chunk sweep and the no-HBM ablation (compute-only ceiling).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2m
mkdir -p $OUT
timeout -k 10 500 python -u tools/k1_probe.py --gb 4 --reps 3 --variants 3:464,3:976,3:400,3:912,3:272,3:784,3:336,3:464:2048,3:464:8192,3:400:8192 > $OUT/sweep4g.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/k1_probe.py --gb 1 --reps 3 --variants 3:464,3:400,3:464:2048,3:400:2048,3:976 > $OUT/sweep1g.log 2>&1 || exit $?
