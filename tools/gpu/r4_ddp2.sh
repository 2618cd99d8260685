#!/bin/bash
# Round 4: BN weight/bias gradients written into the bucket views (no reducer / gather copies).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_a_comm.py tests/test_gpu_wgrad.py \
   tests/test_gpu_bnact.py tests/test_gpu_engine.py > gpurun_out/r4_ddp2_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r4_ddp2_tests.log; [ $rc -eq 0 ] || exit 1
O=gpurun_out/r4_ddp2.txt; : > $O
for i in 1 2; do
for cfg in "ddp --surface ddp" "engine --surface engine"; do
  set -- $cfg; tag=$1; shift 1
  timeout -k 10 300 python bench.py --steps 30 --warmup 12 --exposed-steps 0 --grace-split off "$@" > gpurun_out/r4_ddp2_$tag.log 2>&1 || { echo "FAILED $tag"; tail -5 gpurun_out/r4_ddp2_$tag.log; exit 1; }
  echo "$tag $(python3 tools/diag/benchline.py gpurun_out/r4_ddp2_$tag.log x)" | tee -a $O
done
done
