#!/bin/bash
# r2r: K1 v3 guided schedule with the '\n' count stored before the next chunk's first line:
# chunk-edge line-number test, full GPU tests, pinned-vs-resident diff, probe, bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2r
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/gpu_tests.log 2>&1 || exit $?
tail -3 $OUT/gpu_tests.log
timeout -k 10 400 python -u tools/diff_paths.py > $OUT/diff.log 2>&1 || exit $?
grep -v amdgpu.ids $OUT/diff.log | head -20
timeout -k 10 300 python -u tools/k1_probe.py --gb 4 --reps 3 --variants 3:464,3:464:2048 > $OUT/probe4g.log 2>&1 || exit $?
grep -v amdgpu.ids $OUT/probe4g.log
TSG_K2_STATS=1 timeout -k 10 300 python -u tools/k1_probe.py --gb 4 --reps 1 > $OUT/k2_stats.log 2>&1 || exit $?
grep k2_stats $OUT/k2_stats.log | cut -c1-600
