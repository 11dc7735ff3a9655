#!/bin/bash
# r3i: CR strip with several tiles per counter claim (TSG_CR_VARIANT 0: 8, 1: 4, 2: 16, 3: 2 KiB waves x 8, 4: 1 = r3h)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3i
mkdir -p $OUT
for v in 0 1 2 3 4; do
  for d in 0.025 0; do
    echo "variant $v" >> $OUT/probe.log
    TSG_CR_VARIANT=$v timeout -k 10 120 python -u tools/cr_probe.py --density $d --reps 4 >> $OUT/probe.log 2>&1 || { cat $OUT/probe.log; exit 1; }
  done
done
grep -v amdgpu.ids $OUT/probe.log
for v in 0; do
  TSG_CR_VARIANT=$v timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_cr_strip.py > $OUT/tests_v$v.log 2>&1 || { tail -30 $OUT/tests_v$v.log; exit 1; }
  tail -1 $OUT/tests_v$v.log
done
