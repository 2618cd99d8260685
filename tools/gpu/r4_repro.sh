#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
GRACE_BN_GRAD_TARGET=0 timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread "tests/test_gpu_wgrad.py::test_topk_graph_with_side_stream_runs" > gpurun_out/r4_repro0.log 2>&1; echo "targets off rc=$?"
AMD_LOG_LEVEL=1 timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread "tests/test_gpu_wgrad.py::test_topk_graph_with_side_stream_runs" > gpurun_out/r4_repro1.log 2>&1; echo "targets on rc=$?"
grep -v "^  File" gpurun_out/r4_repro1.log | grep -i -B2 -A2 "error\|abort\|fail\|assert" | head -40
exit 0
