#!/bin/bash
# r3j: CR strip with tiles ordered by workgroup index (TSG_CR_VARIANT 5: 4 KiB waves, 6: 2 KiB waves), 1 GB first.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3j
mkdir -p $OUT
TSG_CR_VARIANT=5 timeout -k 5 60 python -u tools/cr_probe.py --density 0.025 --reps 3 --gb 1 >> $OUT/probe.log 2>&1 || { cat $OUT/probe.log; exit 1; }
for v in 5 6; do
  for d in 0.025 0; do
    echo "variant $v" >> $OUT/probe.log
    TSG_CR_VARIANT=$v timeout -k 5 60 python -u tools/cr_probe.py --density $d --reps 4 >> $OUT/probe.log 2>&1 || { cat $OUT/probe.log; exit 1; }
  done
done
grep -v amdgpu.ids $OUT/probe.log
for v in 5 6; do
  TSG_CR_VARIANT=$v timeout -k 5 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_cr_strip.py > $OUT/tests_v$v.log 2>&1 || { tail -30 $OUT/tests_v$v.log; exit 1; }
  tail -1 $OUT/tests_v$v.log
done
