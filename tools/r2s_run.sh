#!/bin/bash
# r2s: K2 grid with one hit per thread (vs 2 / 4), v3 chunk by launch size (2 KiB at >= 2 GiB): probe + bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s
mkdir -p $OUT
for h in 4 2 1; do
  TSG_K2_HITS_PER_THREAD=$h timeout -k 10 200 python -u tools/k1_probe.py --gb 4 --reps 3 > $OUT/probe4g_h$h.log 2>&1 || exit $?
done
timeout -k 10 300 python -u tools/k1_probe.py --gb 1.4 --reps 3 --variants 3:464:1024,3:464:2048 > $OUT/probe1g.log 2>&1 || exit $?
grep -v amdgpu.ids $OUT/probe4g_h*.log $OUT/probe1g.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_stress.py tests/test_gpu_parity.py > $OUT/gpu_tests.log 2>&1 || exit $?
tail -2 $OUT/gpu_tests.log
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.log || exit $?
cat $OUT/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench -- python3 bench.py --no-cpu-baseline --no-resident --steps 3 > $OUT/bench_prof.json 2> $OUT/bench_prof.log || exit $?
