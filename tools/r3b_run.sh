#!/bin/bash
# r3b: v3 with 64-byte warm-up: variant/stress GPU tests, probe at 1.4 / 4 GB with 1 KiB and 2 KiB chunks.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3b
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_stress.py tests/test_gpu_parity.py > $OUT/gpu_tests.log 2>&1 || exit $?
tail -2 $OUT/gpu_tests.log
for gb in 1.4 4; do
  timeout -k 10 200 python -u tools/k1_probe.py --gb $gb --reps 4 --variants 3:464:1024,3:464:2048 > $OUT/probe_$gb.log 2>&1 || exit $?
  grep -v amdgpu.ids $OUT/probe_$gb.log | cut -c1-200
done
