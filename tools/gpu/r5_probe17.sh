#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=gpurun_out/probe17; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_bnact.py tests/test_gpu_wgrad.py tests/test_gpu_a_comm.py -x -q -W "error:The AccumulateGrad node's stream:UserWarning" --timeout 250 --timeout-method thread > $D/tests.log 2>&1
echo "tests rc=$?"; grep -E "passed|failed|^E  " $D/tests.log | head -6
