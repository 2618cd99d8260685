#!/bin/bash
# Is the DDP-only BN gradient error a race with the reducer's collective stream?  gloo vs RCCL for
# the same pinned configuration, then a kernel trace of the failing RCCL run.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; mkdir -p gpurun_out/ddprace
D=gpurun_out/ddprace
timeout -k 10 100 python -u tools/gpu/ddp_fp64_diag.py --tag gloo --backend gloo --force dgrad=mfma_t2 --modes ddp_off,ddp_on,plain_on > $D/gloo.json 2> $D/gloo.err || exit 1
timeout -k 10 100 python -u tools/gpu/ddp_fp64_diag.py --tag nccl --force dgrad=mfma_t2 --modes ddp_off,ddp_on,plain_on > $D/nccl.json 2> $D/nccl.err || exit 1
grep -o '"tag": "[a-z]*", "mode": "[a-z_]*"\|"max_param_rel_err": [0-9.e+-]*' $D/gloo.json $D/nccl.json
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $D/prof -o trace -- python -u tools/gpu/ddp_fp64_diag.py --tag prof --force dgrad=mfma_t2 --modes ddp_off > $D/prof.json 2> $D/prof.err
echo "prof rc=$?"; grep -o '"max_param_rel_err": [0-9.e+-]*' $D/prof.json
find $D/prof -name "*.csv" | head
