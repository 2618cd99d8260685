#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_wgrad.py > gpurun_out/r3_defer_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r3_defer_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/r3_cfgs.sh "side A=1" "defer GRACE_WGRAD_DEFER=1" "side_b A=1" "defer_b GRACE_WGRAD_DEFER=1"
