#!/bin/bash
# Round 4: the new xGMI all-reduce / second-capture tests, then the compressed-config sweep.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_xgmi.py tests/test_gpu_wgrad.py > gpurun_out/r4_t3.log 2>&1 || { tail -30 gpurun_out/r4_t3.log; exit 1; }
tail -2 gpurun_out/r4_t3.log
bash tools/gpu/r4_sweep2.sh
