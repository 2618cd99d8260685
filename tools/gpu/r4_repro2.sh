#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
AMD_LOG_LEVEL=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_a_comm.py tests/test_gpu_wgrad.py > gpurun_out/r4_repro2.log 2>&1; echo "rc=$?"
grep -E "PASSED|FAILED|ERROR" gpurun_out/r4_repro2.log | tail -5
grep -v "^  File" gpurun_out/r4_repro2.log | grep -i -B3 -A3 "error\|abort\|assert" | grep -v "^--$" | head -40
exit 0
