#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_bnact.py tests/test_gpu_wgrad.py tests/test_gpu_pool.py > gpurun_out/r3_bnfwd_tests.log 2>&1; rc=$?
tail -1 gpurun_out/r3_bnfwd_tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r3_bnfwd_tests.log | head -20; exit $rc; }
bash tools/gpu/r3_cfgs.sh "fwdatom A=1" "fwdtree GRACE_BN_FWD_ATOMIC=0" "fwdatom_b A=1" "fwdtree_b GRACE_BN_FWD_ATOMIC=0"
