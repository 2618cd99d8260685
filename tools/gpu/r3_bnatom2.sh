#!/bin/bash
# Round 3: BN GPU tests, then the headline A/B of the atomic-totals chunk threshold and the
# bucket-direct weight gradients.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_bnact.py tests/test_gpu_wgrad.py > gpurun_out/r3_bnatom2_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r3_bnatom2_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/r3_ab.sh "base A=1" "atom32 GRACE_BN_ATOMIC_CHUNKS=32" "atom100 GRACE_BN_ATOMIC_CHUNKS=100" "nodirect GRACE_WGRAD_DIRECT=0"
