#!/bin/bash
# HBM traffic of K1 from FETCH_SIZE, calibrated on K1's own access pattern
# (run on the GPU box from the repo root; one rocprofv3 --pmc pass per run).
#   tools/pmc_traffic.sh OUTDIR [bench args...]
# then: python tools/pmc_traffic.py OUTDIR > profiles/<round>_traffic.json
set -o pipefail
OUT=${1:-gpurun_out/traffic}; shift
ARGS=${@:---steps 1 --warmup 0}
ROOT=$(pwd)
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $ROOT/$OUT/calib -o calib -- \
  $ROOT/tools/calib_fetch 4 > $ROOT/$OUT/calib.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $ROOT/$OUT/k1 -o k1 -- \
  python3 $ROOT/bench.py $ARGS --no-cpu-baseline > $ROOT/$OUT/k1.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $ROOT/$OUT/k1w -o k1w -- \
  python3 $ROOT/bench.py $ARGS --no-cpu-baseline > $ROOT/$OUT/k1w.log 2>&1 || exit $?
