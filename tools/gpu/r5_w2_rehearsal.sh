#!/bin/bash
# W = 2 whole-step-graph rehearsals of the five BASELINE pipelines: two ranks SHARING one MI355X,
# gloo bootstrap, every GRACE collective on the xGMI one-shot comm (plumbing rehearsal, not a
# scaling number).  Usage: r5_w2_rehearsal.sh [workload ...]
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=gpurun_out/w2; mkdir -p $D
WLS=${@:-resnet50_topk resnet50_dgc vgg16_powersgd lstm_efsignsgd bert_qsgd}
for wl in $WLS; do
  cap=16; [ $wl = bert_qsgd ] && cap=160; [ $wl = vgg16_powersgd ] && cap=32
  timeout -k 10 600 python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29600 + RANDOM % 200)) bench.py --gpus 2 --backend gloo --workload $wl --steps 10 --warmup 6 \
    --xgmi-capacity-mb $cap --grace-split off --exposed-steps 1 > $D/$wl.json 2> $D/$wl.err &
  pid=$!
  while kill -0 $pid 2>/dev/null; do sleep 30; echo "  [$wl running $(date +%T)]"; done
  wait $pid; rc=$?
  echo "$wl rc=$rc $(grep -o '"value": [0-9.]*\|"hip_graph": "[^"]*"\|"comm": "[^"]*"\|"final_loss": [^,]*' $D/$wl.json | tr '\n' ' ')"
  [ $rc -eq 0 ] || { tail -5 $D/$wl.err; exit 1; }
done
