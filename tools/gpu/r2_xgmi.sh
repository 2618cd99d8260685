#!/bin/bash
# One-shot xGMI all-gather: W=2 ranks sharing the box's GPU (IPC handles, generation protocol,
# graph replay, Top-K engine), then the single-rank bench through the xgmi comm.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_xgmi.py -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/xgmi_tests.log 2>&1; rc=$?; tail -8 gpurun_out/xgmi_tests.log; exit $rc
