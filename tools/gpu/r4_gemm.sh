#!/bin/bash
# Round 4: GEMM block-order change -- numerics, per-layer implicit GEMM timings, headline.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_conv3x3.py tests/test_gpu_bnconv.py > gpurun_out/r4_g_t.log 2>&1 || { tail -30 gpurun_out/r4_g_t.log; exit 1; }
tail -1 gpurun_out/r4_g_t.log
timeout -k 10 300 python tools/gpu/conv3_bench.py > gpurun_out/r4_conv3_bench3.txt 2>&1 || { tail -20 gpurun_out/r4_conv3_bench3.txt; exit 1; }
grep wgrad gpurun_out/r4_conv3_bench3.txt | cut -c1-150; tail -1 gpurun_out/r4_conv3_bench3.txt
for i in 1 2; do timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/r4_g_b$i.log 2>&1 || { tail -20 gpurun_out/r4_g_b$i.log; exit 1; }; grep -o '"value": [0-9.]*' gpurun_out/r4_g_b$i.log; done
