#!/bin/bash
# fp32 BN: GPU tests, then per-shape graph-timed totals under grid-shape knobs (one process
# per setting: the knobs are read once), then the headline bench with the default.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bnact.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/bn_tests.log 2>&1; rc=$?; tail -2 gpurun_out/bn_tests.log; [ $rc -eq 0 ] || exit $rc
run() { echo "== $*"; env "$@" timeout -k 10 200 python benchmarks/bnact_bench.py --dtype fp32 > gpurun_out/bnk.txt 2>&1 || { tail -5 gpurun_out/bnk.txt; return 1; }
  grep -E "total per step" gpurun_out/bnk.txt; }
run X=1 && cp gpurun_out/bnk.txt gpurun_out/bnk_default.txt &&
run GRACE_BN_ONE_LEVEL=64 && cp gpurun_out/bnk.txt gpurun_out/bnk_one64.txt &&
run GRACE_BN_ONE_LEVEL=64 GRACE_BN_TARGET_BLOCKS=256 &&
run GRACE_BN_ONE_LEVEL=64 GRACE_BN_VPT_MIN=8 GRACE_BN_VPT_MAX=32 && cp gpurun_out/bnk.txt gpurun_out/bnk_one64_v8.txt &&
run GRACE_BN_TARGET_BLOCKS=256 GRACE_BN_VPT_MAX=32 &&
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench_bn.log 2>&1 && tail -1 gpurun_out/bench_bn.log | cut -c1-200 &&
GRACE_BN_ONE_LEVEL=64 timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench_bn1.log 2>&1 && tail -1 gpurun_out/bench_bn1.log | cut -c1-200
