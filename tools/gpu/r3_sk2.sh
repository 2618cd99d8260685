#!/bin/bash
# Sketch: fence-free encode finisher; encode cost probe (chunk / q / segment structure)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONUNBUFFERED=1; mkdir -p gpurun_out
true \
  > gpurun_out/sk2_tests.log 2>&1 || { tail -30 gpurun_out/sk2_tests.log; exit 1; }
tail -1 gpurun_out/sk2_tests.log
timeout -k 10 200 python benchmarks/grace_kernels.py --pipeline sketch --iters 30 --bucket-mb 128 > gpurun_out/sk2_bench.log 2>&1 || exit 1
tail -1 gpurun_out/sk2_bench.log
timeout -k 10 300 python tools/diag/sketch_encode_probe.py > gpurun_out/sk2_probe.log 2>&1; rc=$?
cat gpurun_out/sk2_probe.log | grep -v amdgpu.ids
exit $rc
