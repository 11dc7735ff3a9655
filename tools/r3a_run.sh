#!/bin/bash
# r3a: K1 launch cost vs size (intercept): 0.01 / 0.1 / 0.5 / 2 / 4 GB resident launches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3a
mkdir -p $OUT
for gb in 0.01 0.1 0.5 2 4; do
  timeout -k 10 200 python -u tools/k1_probe.py --gb $gb --reps 4 > $OUT/probe_$gb.log 2>&1 || exit $?
  echo "$gb $(grep -v amdgpu.ids $OUT/probe_$gb.log | cut -c1-110)"
done
