#!/bin/bash
# r2u: v3 guided schedule with 0/1/2/4 grid rounds of short ranges at launch sizes 0.5, 1.4 and 4 GB.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2u
mkdir -p $OUT
for gb in 0.5 1.4 4; do
  for r in 0 1 2 4; do
    TSG_K1_TAIL_ROUNDS=$r timeout -k 10 200 python -u tools/k1_probe.py --gb $gb --reps 3 > $OUT/probe_${gb}_r$r.log 2>&1 || exit $?
  done
done
for f in $OUT/probe_*.log; do echo "$f $(grep -v amdgpu.ids $f | cut -c1-120)"; done
