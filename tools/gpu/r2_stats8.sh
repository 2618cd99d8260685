#!/bin/bash
# 8-row buffer-load BN statistics: BN tests, per-shape fp32 totals, headline fp32 bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bnact.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/stats8_tests.log 2>&1; rc=$?; tail -2 gpurun_out/stats8_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python benchmarks/bnact_bench.py --dtype fp32 > gpurun_out/bnk_stats8.txt 2>&1 && grep "total per step" gpurun_out/bnk_stats8.txt &&
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench_stats8.log 2>&1 && tail -1 gpurun_out/bench_stats8.log | cut -c1-200
