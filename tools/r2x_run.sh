#!/bin/bash
# r2x: geometric tail segments (config 3 / config 5 pinned path), NUMA binding, config 4 streaming mode,
# new GPU tests (geometric tail, two gloo ranks with engines).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2x
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_stress.py tests/test_multi_rank.py tests/test_layer_tar.py > $OUT/gpu_tests.log 2>&1 || exit $?
tail -2 $OUT/gpu_tests.log
timeout -k 10 600 python -u bench.py --config 3 --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.log || exit $?
cat $OUT/bench_c3.log
timeout -k 10 600 python -u bench.py --config 5 --gb 2 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.log || exit $?
cat $OUT/bench_c5.log
timeout -k 10 700 python -u bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline --no-resident > $OUT/bench_c4.json 2> $OUT/bench_c4.log || exit $?
cat $OUT/bench_c4.log
