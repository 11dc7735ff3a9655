#!/bin/bash
# r3m: K1 FETCH_SIZE traffic with 128-byte register lines (TSG_K1_ABL=272: each lane consumes a whole
# 128-B cache line at once) against the default 64-byte lines (464), same bench layout.
set -o pipefail
cd $GRAFT_REPO_ROOT
TSG_K1_ABL=272 bash tools/pmc_traffic.sh gpurun_out/r3m/t272 --steps 1 --warmup 0 --no-resident || exit $?
bash tools/pmc_traffic.sh gpurun_out/r3m/t464 --steps 1 --warmup 0 --no-resident || exit $?
echo done
