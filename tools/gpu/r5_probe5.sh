#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=gpurun_out/probe5; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_gpu_xgmi.py tests/test_gpu_a_comm.py -x -v --timeout 300 --timeout-method thread -k "not plain_ddp" > $D/xgmi.log 2>&1
echo "xgmi rc=$?"; grep -E "PASS|FAIL|ERROR|passed|failed" $D/xgmi.log | tail -30
