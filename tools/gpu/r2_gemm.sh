#!/bin/bash
# f32 MFMA GEMM / 1x1 conv: GPU tests, then per-layer timing vs MIOpen (+ QSGD/sketch tests).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_sketch.py tests/test_gpu_compressors.py -x -q --timeout 120 --timeout-method thread > gpurun_out/convtests.log 2>&1; rc=$?
tail -15 gpurun_out/convtests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python -u benchmarks/conv_bench.py > gpurun_out/conv_bench2.txt 2>&1 || { tail -20 gpurun_out/conv_bench2.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/conv_bench2.txt
