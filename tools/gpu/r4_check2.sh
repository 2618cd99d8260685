#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_conv3x3.py tests/test_gpu_bnconv.py tests/test_gpu_bnact.py tests/test_gpu_sparse_decode.py tests/test_gpu_compressors.py tests/test_gpu_pool.py > gpurun_out/r4_c2_t.log 2>&1 || { tail -30 gpurun_out/r4_c2_t.log; exit 1; }
tail -1 gpurun_out/r4_c2_t.log
for i in 1 2; do timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/r4_c2_b$i.log 2>&1 || { tail -20 gpurun_out/r4_c2_b$i.log; exit 1; }; grep -o '"value": [0-9.]*' gpurun_out/r4_c2_b$i.log; done
