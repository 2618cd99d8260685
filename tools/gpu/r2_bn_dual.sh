#!/bin/bash
# Dual-output BN (block-output gradients summed inside the BN backward): BN GPU tests, headline
# bench fp32 + bf16, per-step kernel table.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bnact.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/bn_tests.log 2>&1; rc=$?; tail -2 gpurun_out/bn_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench_dual.log 2>&1 && tail -1 gpurun_out/bench_dual.log | cut -c1-200 &&
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --dtype bf16 > gpurun_out/bench_dual_bf16.log 2>&1 && tail -1 gpurun_out/bench_dual_bf16.log | cut -c1-200 &&
bash tools/gpu/r2_bn_grid.sh dual > /dev/null && head -40 gpurun_out/prof_dual_steps.txt
