#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
O=gpurun_out/r4_ddp3.txt; : > $O
for i in 1 2; do
for cfg in "ddp_side GRACE_DDP_SIDE_WGRAD=1 --surface ddp" "ddp_inline GRACE_DDP_SIDE_WGRAD=0 --surface ddp"; do
  set -- $cfg; tag=$1; envv=$2; shift 2
  env $envv timeout -k 10 300 python bench.py --steps 30 --warmup 12 --exposed-steps 0 --grace-split off "$@" > gpurun_out/r4_ddp3_$tag.log 2>&1 || { echo "FAILED $tag"; tail -5 gpurun_out/r4_ddp3_$tag.log; exit 1; }
  echo "$tag $(python3 tools/diag/benchline.py gpurun_out/r4_ddp3_$tag.log x)" | tee -a $O
done
done
GRACE_DDP_SIDE_WGRAD=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_a_comm.py > gpurun_out/r4_ddp3_tests.log 2>&1; echo "side tests rc=$?"; tail -1 gpurun_out/r4_ddp3_tests.log
