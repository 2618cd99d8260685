#!/bin/bash
# Fused BN+ReLU+maxpool stem: BN/pool GPU tests, headline fp32 + bf16 benches, per-step kernel table.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bnact.py tests/test_gpu_pool.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/stem_tests.log 2>&1; rc=$?; tail -2 gpurun_out/stem_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench_stem.log 2>&1 && tail -1 gpurun_out/bench_stem.log | cut -c1-200 &&
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --dtype bf16 > gpurun_out/bench_stem_bf16.log 2>&1 && tail -1 gpurun_out/bench_stem_bf16.log | cut -c1-200 &&
bash tools/gpu/r2_bn_grid.sh stem > /dev/null && grep -E "pool|window|grace_amd" gpurun_out/prof_stem_steps.txt
