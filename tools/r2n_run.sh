#!/bin/bash
# r2n: K1 v4 (two streams per lane): variant-agreement GPU tests, then v3 vs v4 probe.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2n
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_stress.py -k "variants and 4-" > $OUT/gpu_tests.log 2>&1 || exit $?
tail -3 $OUT/gpu_tests.log
timeout -k 10 300 python -u tools/k1_probe.py --gb 4 --reps 3 --variants 3:464,4,4::2048,4::8192 > $OUT/probe4g.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/k1_probe.py --gb 1 --reps 3 --variants 3:464,4,4::2048 > $OUT/probe1g.log 2>&1 || exit $?
grep -v amdgpu.ids $OUT/probe4g.log $OUT/probe1g.log
