#!/bin/bash
# Full GPU check on the box: GPU tests, smoke, default bench (CPU baseline +
# parity), rocprofv3 kernel-trace stats of a bench run.
#   tools/gpu_full.sh TAG
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
ROOT=$(pwd)
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit $?
tail -2 $OUT/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
cat $OUT/smoke.log
timeout -k 10 400 python bench.py --json-out $OUT/bench.json > $OUT/bench.out 2> $OUT/bench.log || exit $?
cat $OUT/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof -o run -- python3 $ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-pcie > $ROOT/$OUT/prof.log 2>&1 || exit $?
cd $ROOT && find $OUT/prof -name '*.db' -o -name '*stats*' | head
