#!/bin/bash
# Round 3: BN backward atomic totals + wgrad straight into the bucket + SGD load batching --
# BN / wgrad / engine / optimizer GPU tests, then the headline A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_bnact.py tests/test_gpu_wgrad.py tests/test_gpu_engine.py tests/test_gpu_conv.py > gpurun_out/r3_bnatom_tests.log 2>&1; rc=$?
tail -4 gpurun_out/r3_bnatom_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/r3_ab.sh "new A=1" "tree GRACE_BN_DETERMINISTIC=1" "nodirect GRACE_WGRAD_DIRECT=0"
