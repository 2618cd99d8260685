#!/bin/bash
# After the capture-mode change (thread-local whenever an RCCL group is up): DDP surface at W = 1
# (an RCCL group of one rank), the engine, and the W = 2 gloo whole-step-graph rehearsal.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=$R/gpurun_out/postcap; mkdir -p $D
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --surface ddp --steps 30 --warmup 10 > $D/ddp$i.json 2> $D/ddp$i.err || { tail -5 $D/ddp$i.err; exit 1; }
  echo "ddp$i $(grep -o '"value": [0-9.]*\|"hip_graph": "[^"]*"' $D/ddp$i.json | tr '\n' ' ')"
done
timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $D/eng.json 2> $D/eng.err || exit 1
echo "engine $(grep -o '"value": [0-9.]*' $D/eng.json)"
bash tools/gpu/r5_w2_rehearsal.sh resnet50_topk
