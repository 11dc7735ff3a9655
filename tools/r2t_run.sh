#!/bin/bash
# r2t: is K1's fixed per-launch cost clock ramp-up?  probe with and without a busy GPU right before each run.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2t
mkdir -p $OUT
for gb in 1.4 4; do
  timeout -k 10 200 python -u tools/k1_probe.py --gb $gb --reps 3 > $OUT/probe_${gb}_cold.log 2>&1 || exit $?
  timeout -k 10 200 python -u tools/k1_probe.py --gb $gb --reps 3 --prewarm-ms 30 > $OUT/probe_${gb}_warm.log 2>&1 || exit $?
done
grep -v amdgpu.ids $OUT/probe_*.log | cut -c1-200
