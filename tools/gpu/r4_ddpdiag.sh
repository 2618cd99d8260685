#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; mkdir -p gpurun_out
T=tests/test_gpu_a_comm.py::test_plain_ddp_resnet_grads_match_inline
for i in 1 2 3 4 5 6; do
  timeout -k 10 120 python -u -m pytest $T -m gpu -q --timeout 100 --timeout-method thread > gpurun_out/diag$i.log 2>&1
  rc=$?; echo "run $i rc=$rc $(grep -E '^E  |passed|failed' gpurun_out/diag$i.log | head -3 | cut -c1-600 | tr '\n' ' ')"
  [ $rc -le 1 ] || exit 1
done
