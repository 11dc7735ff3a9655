#!/bin/bash
# r3e: CR strip kernel timing and per-kernel rocprof split.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r3e}
mkdir -p $OUT
timeout -k 10 200 python -u tools/cr_probe.py --density 0.025 > $OUT/probe.log 2>&1 || { cat $OUT/probe.log; exit 1; }
timeout -k 10 200 python -u tools/cr_probe.py --density 0 >> $OUT/probe.log 2>&1 || { cat $OUT/probe.log; exit 1; }
timeout -k 10 200 python -u tools/cr_probe.py --density 0.5 --gb 4 >> $OUT/probe.log 2>&1 || { cat $OUT/probe.log; exit 1; }
cat $OUT/probe.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o cr -- python3 tools/cr_probe.py --density 0.025 > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 1; }
python tools/prof_summary.py $OUT/prof/cr_results.db > $OUT/kernel_stats.csv && grep tsg_cr $OUT/kernel_stats.csv | cut -c1-60,200-400
