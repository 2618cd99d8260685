#!/bin/bash
# W=2 ranks on the one GPU of a gpurun box (gloo carries cuda:0 payloads): every codec and the
# bucketed engine in a real multi-rank exchange.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_multirank.log 2>&1; rc=$?; tail -6 gpurun_out/gpu_multirank.log; exit $rc
