#!/bin/bash
# Round 4: DDP comm-hook surface with side-stream weight gradients for DDP parameters (stable
# buckets only), A/B against in-line, and the engine on the same box.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_a_comm.py tests/test_gpu_wgrad.py > gpurun_out/r4_ddp_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r4_ddp_tests.log; [ $rc -eq 0 ] || exit 1
O=gpurun_out/r4_ddp.txt; : > $O
for i in 1 2; do
for cfg in "ddp_side GRACE_DDP_SIDE_WGRAD=1 --surface ddp" "ddp_inline GRACE_DDP_SIDE_WGRAD=0 --surface ddp" "engine X=1 --surface engine"; do
  set -- $cfg; tag=$1; envv=$2; shift 2
  env $envv timeout -k 10 300 python bench.py --steps 30 --warmup 12 --exposed-steps 0 --grace-split off "$@" > gpurun_out/r4_ddp_$tag.log 2>&1 || { echo "FAILED $tag"; tail -5 gpurun_out/r4_ddp_$tag.log; exit 1; }
  echo "$tag $(python3 tools/diag/benchline.py gpurun_out/r4_ddp_$tag.log x) $(grep -o '"surface": "[^"]*"' gpurun_out/r4_ddp_$tag.log)" | tee -a $O
done
done
