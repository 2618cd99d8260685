#!/bin/bash
# the fp64 plain-DDP test, in fresh processes (the r4 flake was per process), plus the forced
# configuration that reproduced the ReLU-kink flip reliably (dgrad=mfma_t2)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=gpurun_out/ddptest; mkdir -p $D
T="tests/test_gpu_a_comm.py -k plain_ddp"
for i in 1 2 3; do
  timeout -k 10 150 python -u -m pytest $T -v -q --timeout 120 --timeout-method thread > $D/run$i.log 2>&1
  rc=$?; echo "run $i rc=$rc $(grep -E '^E  |passed|failed' $D/run$i.log | head -2 | cut -c1-300 | tr '\n' ' ')"
  [ $rc -le 1 ] || exit 1
done
