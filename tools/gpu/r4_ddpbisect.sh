#!/bin/bash
# Which fused path makes plain-DDP resnet18 grads differ between wgrad stream on/off?
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; mkdir -p gpurun_out
T=tests/test_gpu_a_comm.py::test_plain_ddp_resnet_grads_match_inline
for cfg in "GRACE_X=0" "GRACE_CONV3X3=0" "GRACE_CONV_BN_STATS=0" "GRACE_CONV_AUTO=0" "GRACE_BN_DZ=0"; do
  env $cfg timeout -k 10 120 python -u -m pytest $T -m gpu -q --timeout 100 --timeout-method thread > gpurun_out/bis.log 2>&1
  rc=$?; echo "$cfg rc=$rc $(grep -E 'assert 0|passed|failed' gpurun_out/bis.log | head -2 | tr '\n' ' ')"
  [ $rc -le 1 ] || exit 1
done
