#!/bin/bash
# BN folds with sc1 loads instead of the acquire: BN GPU tests, headline bench, per-layer trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bnact.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/bn_tests.log 2>&1; rc=$?; tail -3 gpurun_out/bn_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench_sc1.log 2>&1 && tail -1 gpurun_out/bench_sc1.log | cut -c1-330 &&
bash tools/gpu/r2_bn_grid.sh sc1 > /dev/null && head -12 gpurun_out/prof_sc1_steps.txt && tail -1 gpurun_out/prof_sc1_bnseq.txt
