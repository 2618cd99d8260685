#!/bin/bash
# Round 4: implicit-GEMM conv + BN hand-off numerics, per-layer A/B vs MIOpen, headline A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_conv3x3.py tests/test_gpu_bnconv.py tests/test_gpu_conv.py > gpurun_out/r4_c3_t.log 2>&1 || { tail -40 gpurun_out/r4_c3_t.log; exit 1; }
tail -2 gpurun_out/r4_c3_t.log
timeout -k 10 300 python tools/gpu/conv3_bench.py > gpurun_out/r4_conv3_bench.txt 2>&1 || { tail -20 gpurun_out/r4_conv3_bench.txt; exit 1; }
cat gpurun_out/r4_conv3_bench.txt
O=gpurun_out/r4_c3_ab.txt; : > $O
ab() { local tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/c3ab_$tag.log 2>&1 || { tail -20 gpurun_out/c3ab_$tag.log; exit 1; }; echo "$tag $(grep -o '"value": [0-9.]*' gpurun_out/c3ab_$tag.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c3ab_$tag.log)" >> $O; tail -1 $O; }
ab new GRACE_X=1
ab no_pro GRACE_BN_PROLOGUE=0
ab no_pro_no_bnepi GRACE_BN_PROLOGUE=0 GRACE_BN_BWD_EPI=0
ab base GRACE_BN_PROLOGUE=0 GRACE_BN_BWD_EPI=0 GRACE_CONV3X3=0
ab new_b GRACE_X=1
