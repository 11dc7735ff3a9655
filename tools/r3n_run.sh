#!/bin/bash
# r3n (round-2 final, rebuilt container): full GPU tests, smoke (with the CRLF smoke files), default bench (config 2),
# rocprof kernel trace of the bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3n
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.log || { tail -20 $OUT/bench.log; exit 1; }
cat $OUT/bench.log
[ -n "$R3N_NOPROF" ] || timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench -- python3 bench.py --no-cpu-baseline --steps 3 > $OUT/bench_prof.json 2> $OUT/bench_prof.log || { tail $OUT/bench_prof.log; exit 1; }
echo done
