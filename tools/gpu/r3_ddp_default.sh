#!/bin/bash
# DDP surface with bench defaults (graph auto -> full) at W = 1, and a W = 2 gloo rehearsal of the
# DDP hook path on one GPU (gloo: eager)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONUNBUFFERED=1; mkdir -p gpurun_out
timeout -k 10 300 python bench.py --surface ddp --steps 30 --warmup 12 > gpurun_out/ddp_default.log 2>&1 || { tail -5 gpurun_out/ddp_default.log; exit 1; }
python3 tools/diag/benchline.py gpurun_out/ddp_default.log ddp_default
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 \
  bench.py --gpus 2 --backend gloo --surface ddp --steps 5 --warmup 3 > gpurun_out/ddp_w2_gloo.log 2>&1 || { tail -8 gpurun_out/ddp_w2_gloo.log; exit 1; }
grep '^{' gpurun_out/ddp_w2_gloo.log | tail -1 | cut -c1-400
