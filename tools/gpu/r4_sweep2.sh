#!/bin/bash
# Round 4 sweep, part 2: the compressed configs (grace split on) after the no-op-capture fix.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
O=gpurun_out/r4_sweep2.txt; : > $O
b() { local tag=$1; shift; timeout -k 10 400 python bench.py --steps 30 --warmup 10 "$@" > gpurun_out/sw4_$tag.log 2>&1 && echo "$tag $(grep '"metric"' gpurun_out/sw4_$tag.log)" >> $O || { echo "FAILED $tag" >> $O; tail -3 gpurun_out/sw4_$tag.log >> $O; exit 1; }; tail -1 $O | cut -c1-200; }
b resnet50_topk
b resnet50_dgc --workload resnet50_dgc
b resnet50_threshold --workload resnet50_threshold
b vgg16_powersgd --workload vgg16_powersgd --steps 20
b lstm_efsignsgd --workload lstm_efsignsgd --steps 40
b bert_qsgd --workload bert_qsgd --steps 20
b resnet50_topk_b
grep -c AccumulateGrad gpurun_out/sw4_resnet50_topk.log || true
