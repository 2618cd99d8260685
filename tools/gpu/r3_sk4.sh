#!/bin/bash
# Sketch: fixed-point integer bin sums in the encode; tests, exchange bench, encode probe, kernel table
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONUNBUFFERED=1; mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sketch.py \
  > gpurun_out/sk4_tests.log 2>&1 || { tail -30 gpurun_out/sk4_tests.log; exit 1; }
tail -1 gpurun_out/sk4_tests.log
timeout -k 10 200 python benchmarks/grace_kernels.py --pipeline sketch --iters 30 --bucket-mb 128 > gpurun_out/sk4_bench.log 2>&1 || exit 1
tail -1 gpurun_out/sk4_bench.log
timeout -k 10 200 python tools/diag/sketch_encode_probe.py > gpurun_out/sk4_probe.log 2>&1 || exit 1
grep "us$" gpurun_out/sk4_probe.log
bash tools/gpu/r3_sketch_prof.sh
