#!/bin/bash
# Round 4: one-launch sparse decode tests + microbench, then the compressed-config sweep.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; mkdir -p gpurun_out
timeout -k 10 200 python tools/gpu/decode_bench.py > gpurun_out/r4_decode_bench.txt 2>&1 || { tail -20 gpurun_out/r4_decode_bench.txt; exit 1; }
cat gpurun_out/r4_decode_bench.txt
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_sparse_decode.py tests/test_gpu_xgmi.py tests/test_gpu_wgrad.py tests/test_gpu_topk.py tests/test_gpu_capacity_graph.py > gpurun_out/r4_dec_t.log 2>&1 || { tail -40 gpurun_out/r4_dec_t.log; exit 1; }
tail -2 gpurun_out/r4_dec_t.log
