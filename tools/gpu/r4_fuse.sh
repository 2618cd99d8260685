#!/bin/bash
# Round 4: BN-in-GEMM fusion numerics + headline A/B, then the decode tests / microbench.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_bnconv.py tests/test_gpu_conv.py tests/test_gpu_conv3x3.py > gpurun_out/r4_fu_t.log 2>&1 || { tail -40 gpurun_out/r4_fu_t.log; exit 1; }
tail -1 gpurun_out/r4_fu_t.log
O=gpurun_out/r4_fuse_ab.txt; : > $O
ab() { local tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/fuab_$tag.log 2>&1 || { tail -20 gpurun_out/fuab_$tag.log; exit 1; }; echo "$tag $(grep -o '"value": [0-9.]*' gpurun_out/fuab_$tag.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fuab_$tag.log)" >> $O; tail -1 $O; }
timeout -k 10 300 python tools/gpu/conv3_bench.py > gpurun_out/r4_conv3_bench2.txt 2>&1 || { tail -20 gpurun_out/r4_conv3_bench2.txt; exit 1; }
tail -3 gpurun_out/r4_conv3_bench2.txt
ab base GRACE_X=1
ab conv3pro GRACE_BN_PROLOGUE=2
ab base_b GRACE_X=1
ab conv3pro_b GRACE_BN_PROLOGUE=2
