#!/bin/bash
# BN reduction-tree change: BN GPU tests, per-shape graph timing, headline bench.
#   gpurun --timeout 900 -- 'bash tools/gpu/bn_fold_check.sh'
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bnact.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/bn_tests.log 2>&1; rc=$?; tail -3 gpurun_out/bn_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python bench.py --steps 30 --warmup 10 > gpurun_out/b_fold.log 2>&1 && tail -1 gpurun_out/b_fold.log | cut -c1-200 &&
timeout -k 10 240 python benchmarks/bnact_bench.py > gpurun_out/bn_shapes.txt 2>&1 && tail -20 gpurun_out/bn_shapes.txt &&
python -c "import grace_amd.ops._native as n; print('spin timeouts', n.lib().bn_spin_timeouts())"
