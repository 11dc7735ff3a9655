#!/bin/bash
# r2w: layer-tar GPU test; config 3 (image layers, incl. the layer-tar feed rate) and config 5 on the pinned path.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2w
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_layer_tar.py tests/test_config3.py > $OUT/gpu_tests.log 2>&1 || exit $?
tail -2 $OUT/gpu_tests.log
timeout -k 10 600 python -u bench.py --config 3 > $OUT/bench_c3.json 2> $OUT/bench_c3.log || exit $?
cat $OUT/bench_c3.log
timeout -k 10 600 python -u bench.py --config 5 --gb 2 > $OUT/bench_c5.json 2> $OUT/bench_c5.log || exit $?
cat $OUT/bench_c5.log
