#!/bin/bash
# Plain-DDP gradient mismatch: every mode vs an fp64 CPU reference, in 4 fresh processes (the
# failure is per process: a timed choice), MIOpen's solver log kept for each.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; mkdir -p gpurun_out/ddpdiag
for i in 1 2 3 4; do
  MIOPEN_ENABLE_LOGGING=1 MIOPEN_LOG_LEVEL=6 timeout -k 10 150 python -u tools/gpu/ddp_fp64_diag.py --tag run$i \
    > gpurun_out/ddpdiag/run$i.json 2> gpurun_out/ddpdiag/run$i.miopen.log
  rc=$?
  echo "run $i rc=$rc"; grep -o '"mode": "[a-z_]*", "loss": [0-9.]*\|"max_param_rel_err": [0-9.e+-]*\|"n": [0-9]*' gpurun_out/ddpdiag/run$i.json | tr '\n' ' '; echo
  [ $rc -eq 0 ] || exit 1
done
