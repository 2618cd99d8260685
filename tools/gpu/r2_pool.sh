#!/bin/bash
# NHWC maxpool: GPU tests, headline fp32 bench, VGG-16 fp32 bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pool.py tests/test_gpu_convact.py tests/test_gpu_bnact.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pool_tests.log 2>&1; rc=$?; tail -2 gpurun_out/pool_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench_pool.log 2>&1 && tail -1 gpurun_out/bench_pool.log | cut -c1-200 &&
timeout -k 10 400 python bench.py --workload vgg16_powersgd --steps 20 --warmup 10 > gpurun_out/bench_vgg_pool.log 2>&1 && tail -1 gpurun_out/bench_vgg_pool.log | cut -c1-200 &&
bash tools/gpu/r2_bn_grid.sh pool > /dev/null && grep -E "max_pool|maxpool|window|grace_amd" gpurun_out/prof_pool_steps.txt
