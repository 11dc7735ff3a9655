#!/bin/bash
# PMC passes for the K1/K2 kernels (run on the GPU box from the repo root).
# Each pass is its own rocprofv3 run (counters are not split over passes).
#   tools/pmc_k1.sh OUTDIR [bench args...]
set -o pipefail
OUT=${1:-gpurun_out/pmc}; shift
ARGS=${@:---gb 2 --steps 1 --warmup 0}
mkdir -p $OUT
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
run() {
  name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $ROOT/$OUT/$name -o $name -- \
    python3 $ROOT/bench.py $ARGS --no-cpu-baseline > $ROOT/$OUT/$name.log 2>&1
}
run p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS && \
run p2 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_LDS && \
run p3 FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT && \
run p4 WRITE_SIZE && \
run p5 SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_IFETCH SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY
