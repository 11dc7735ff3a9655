set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u tools/k1_probe.py --gb 4 --reps 3 --variants 1:0:4096,3:208:2048,3:464:2048,3:336:2048,3:464:4096,3:466:2048 > gpurun_out/r2d_k1_defer.log 2>&1 && \
TSG_K1_VARIANT=3 TSG_K1_ABL=464 TSG_K1_CHUNK=2048 timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r2d_v3_tests.log 2>&1
