#!/bin/bash
# Kernel trace + PMC passes over tools/k1_probe.py (HBM-resident batch, K1+K2 only).
# Each pass is its own rocprofv3 run (counters are not split over passes).
#   tools/pmc_probe.sh OUTDIR [k1_probe args...]        (from the repo root, on the GPU box)
set -o pipefail
OUT=${1:-gpurun_out/pmc}; shift
ARGS=${@:---gb 4 --reps 3}
ROOT=$(pwd)
mkdir -p $ROOT/$OUT
cd /tmp && export TMPDIR=/tmp
run() {
  name=$1; shift
  timeout -s KILL 150 rocprofv3 "$@" --output-format csv -d $ROOT/$OUT/$name -o $name -- \
    python3 $ROOT/tools/k1_probe.py $ARGS > $ROOT/$OUT/$name.log 2>&1
}
run trace --kernel-trace --stats && \
run p1 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS && \
run p2 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_IFETCH && \
run p3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE && \
run p4 --pmc WRITE_SIZE && \
run p5 --pmc SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES SQ_INSTS_VALU
