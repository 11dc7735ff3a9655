#!/bin/bash
# K1's L2 -> memory read requests by size and by destination (one rocprofv3
# --pmc pass, four TCC counters): TCC_EA0_RDREQ (all), _64B / _128B (request
# size), _DRAM (destined for the local memory side: HBM or the Infinity
# Cache in front of it, which no counter on this ROCm separates).
#   tools/pmc_dram.sh OUTDIR [bench args...]
set -o pipefail
OUT=${1:-gpurun_out/dram}; shift
ARGS=${@:---steps 1 --warmup 0}
ROOT=$(pwd)
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_DRAM_sum \
  --output-format csv -d $ROOT/$OUT/dram -o dram -- \
  python3 $ROOT/bench.py $ARGS --no-cpu-baseline > $ROOT/$OUT/dram.log 2>&1 || exit $?
