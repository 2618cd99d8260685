#!/bin/bash
# Sketch: batched slot loads in the selection scans; tests, exchange bench, kernel table
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONUNBUFFERED=1; mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sketch.py \
  > gpurun_out/sk5_tests.log 2>&1 || { tail -30 gpurun_out/sk5_tests.log; exit 1; }
tail -1 gpurun_out/sk5_tests.log
timeout -k 10 200 python benchmarks/grace_kernels.py --pipeline sketch --iters 30 --bucket-mb 128 > gpurun_out/sk5_bench.log 2>&1 || exit 1
tail -1 gpurun_out/sk5_bench.log
bash tools/gpu/r3_sketch_prof.sh
