#!/bin/bash
# Round 4: implicit-GEMM 3x3 conv numerics + per-layer A/B vs MIOpen, then headline bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_conv3x3.py > gpurun_out/r4_c3_t.log 2>&1 || { tail -40 gpurun_out/r4_c3_t.log; exit 1; }
tail -2 gpurun_out/r4_c3_t.log
timeout -k 10 300 python tools/gpu/conv3_bench.py > gpurun_out/r4_conv3_bench.txt 2>&1 || { tail -20 gpurun_out/r4_conv3_bench.txt; exit 1; }
cat gpurun_out/r4_conv3_bench.txt
timeout -k 10 400 python bench.py --steps 30 --warmup 10 > gpurun_out/r4_c3_bench.log 2>&1 || { tail -20 gpurun_out/r4_c3_bench.log; exit 1; }
grep '"metric"' gpurun_out/r4_c3_bench.log | cut -c1-400
