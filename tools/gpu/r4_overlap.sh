#!/bin/bash
# Round 4: --overlap on vs off at W = 2 (two ranks share the one GPU; gloo bootstraps, the
# exchange runs on the xGMI one-shot comm inside the whole-step graph) -- a REHEARSAL of the
# overlap decision, not a scaling number.  Top-K (small payload) and None/Allreduce (102 MB).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
O=gpurun_out/r4_overlap.txt; : > $O
port=29611
run() { local tag=$1; shift; port=$((port+1));
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port \
    bench.py --gpus 2 --backend gloo --comm auto --graph full --xgmi-capacity-mb 128 --steps 20 --warmup 6 "$@" \
    > gpurun_out/ov_$tag.log 2>&1 && echo "$tag $(grep '"metric"' gpurun_out/ov_$tag.log)" >> $O \
    || { echo "FAILED $tag" >> $O; tail -5 gpurun_out/ov_$tag.log >> $O; exit 1; }; tail -1 $O | cut -c1-160; }
run topk_off --overlap off
run topk_on --overlap on
run none_off --workload resnet50_none --overlap off
run none_on --workload resnet50_none --overlap on
