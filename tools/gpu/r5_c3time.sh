#!/bin/bash
# 3x3 implicit-GEMM numerics (canary OOB + conv3x3 + GEMM tests), then per-layer timings vs MIOpen.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=gpurun_out/c3time; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_oob.py tests/test_gpu_conv3x3.py tests/test_gpu_conv.py tests/test_gpu_bnconv.py -x -q \
  --timeout 250 --timeout-method thread > $D/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|^E  " $D/tests.log | head -6; [ $rc -eq 0 ] || exit $rc
for cfg in "32 256 14 14 1 4 1" "32 256 14 14 1 2 1" "32 256 14 14 1 -1 1" "32 512 7 7 1 2 4" "32 512 7 7 1 4 2" "32 512 7 7 1 -1 1" "32 128 28 28 1 2 1" "32 128 28 28 1 -1 1"; do
  timeout -k 10 60 python3 tools/gpu/c3_pmc_one.py $cfg 20 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 400 python -u tools/gpu/conv3_bench.py > $D/conv3_bench.txt 2>&1 || exit 1
grep -v amdgpu.ids $D/conv3_bench.txt | cut -c1-250
timeout -k 10 300 python -u -m pytest tests/test_gpu_compressors.py tests/test_gpu_capacity_graph.py -x -q -k "threshold or capacity" \
  --timeout 250 --timeout-method thread > $D/thr_tests.log 2>&1 || { tail -20 $D/thr_tests.log; exit 1; }
grep -E "passed|failed" $D/thr_tests.log | tail -1
timeout -k 10 200 python -u benchmarks/grace_kernels.py --pipeline threshold --iters 30 --bucket-mb 128 2>&1 | grep -v amdgpu.ids | tail -2
