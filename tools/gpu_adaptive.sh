set -o pipefail
mkdir -p gpurun_out/r1o
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r1o/gpu_tests.log 2>&1 || exit $?
tail -2 gpurun_out/r1o/gpu_tests.log
tools/gpu_pieces.sh r1o 1:0.5 2:0.7 || exit $?
TSG_K1_ADAPTIVE=0 tools/gpu_pieces.sh r1o_fixed 1:0.5 2:0.7
