#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_bnact.py > gpurun_out/r3_bnatom3_tests.log 2>&1; rc=$?
tail -1 gpurun_out/r3_bnatom3_tests.log; [ $rc -eq 0 ] || exit $rc
GRACE_BN_ATOMIC_CHUNKS=100000 timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_bnact.py -k "fp32 or dual or maxpool or atomic" > gpurun_out/r3_bnatom3_tests2.log 2>&1; rc=$?
tail -1 gpurun_out/r3_bnatom3_tests2.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/r3_cfgs.sh "base A=1" "atom32 GRACE_BN_ATOMIC_CHUNKS=32" "atom128 GRACE_BN_ATOMIC_CHUNKS=128" "atomall GRACE_BN_ATOMIC_CHUNKS=100000" "base_b A=1"
