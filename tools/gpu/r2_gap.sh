#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pool.py tests/test_gpu_bnact.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/gap_tests.log 2>&1; rc=$?; tail -2 gpurun_out/gap_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench_gap.log 2>&1 && tail -1 gpurun_out/bench_gap.log | cut -c1-200 &&
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --dtype bf16 > gpurun_out/bench_gap_bf16.log 2>&1 && tail -1 gpurun_out/bench_gap_bf16.log | cut -c1-200 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_gap.log 2>&1 && tail -1 gpurun_out/smoke_gap.log
