#!/bin/bash
# r2o: v3 with integer LDS transition addresses (one VALU per byte less) vs the pointer form; v4 at 512 threads.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2o
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_stress.py -k "variants" > $OUT/gpu_tests.log 2>&1 || exit $?
tail -3 $OUT/gpu_tests.log
timeout -k 10 300 python -u tools/k1_probe.py --gb 4 --reps 3 --variants 3:464,3:1488,3:976,4:0::512/1,4 > $OUT/probe4g.log 2>&1 || exit $?
grep -v amdgpu.ids $OUT/probe4g.log
