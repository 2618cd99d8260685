#!/bin/bash
# Round 4: fp32 single-launch BN kernels -- correctness, per-shape timing, headline A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bnact.py > gpurun_out/r4_bnfused_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r4_bnfused_tests.log; [ $rc -eq 0 ] || exit 1
O=gpurun_out/r4_bnfused_bench.txt; : > $O
for cfg in "GRACE_BN_FUSED_F32=1" "GRACE_BN_FUSED_F32=0"; do
  echo "== $cfg" >> $O; env $cfg timeout -k 10 200 python benchmarks/bnact_bench.py --dtype fp32 --iters 20 >> $O 2>&1 || { echo FAILED >> $O; exit 1; }
done
for cfg in "GRACE_BN_FUSED_F32=1" "GRACE_BN_FUSED_F32=0" "GRACE_BN_FUSED_F32=1" "GRACE_BN_FUSED_F32=0"; do
  env $cfg timeout -k 10 300 python bench.py --steps 30 --warmup 10 --exposed-steps 0 --grace-split off > gpurun_out/r4_bf.log 2>&1 || { echo "bench FAILED $cfg"; tail -5 gpurun_out/r4_bf.log; exit 1; }
  echo "$cfg $(python3 tools/diag/benchline.py gpurun_out/r4_bf.log x)" | tee -a $O
done
grep -E "^ +[0-9]|total" $O | head -40
