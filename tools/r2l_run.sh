#!/bin/bash
# r2l: K1 v3 ablations (what bounds K1), PMC counters of K1/K2 on a 4 GB
# resident launch, and FETCH_SIZE/WRITE_SIZE traffic of the bench layout.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2l
mkdir -p $OUT
timeout -k 10 400 python -u tools/k1_probe.py --gb 4 --reps 3 --variants 3:464,3:496,3:468,3:466,3:472,3:465,3:208 > $OUT/ablation.log 2>&1 || exit $?
bash tools/pmc_probe.sh $OUT/pmc --gb 4 --reps 2 || exit $?
bash tools/pmc_traffic.sh $OUT/traffic --steps 1 --warmup 0 --no-resident || exit $?
