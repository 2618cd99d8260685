#!/bin/bash
# Round 4 sweep: every BASELINE config at W = 1 on the current state (fp32 headline precision),
# each with its None/Allreduce reference, plus the GRACE exchange microbenchmarks.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
O=gpurun_out/r4_sweep.txt; : > $O
for p in topk dgc threshold powersgd qsgd efsignsgd sketch; do
  timeout -k 10 200 python benchmarks/grace_kernels.py --pipeline $p --iters 20 --bucket-mb 128 2>/dev/null | tail -1 >> $O || echo "grace_kernels $p failed" >> $O
done
b() { local tag=$1; shift; timeout -k 10 400 python bench.py --steps 30 --warmup 10 "$@" > gpurun_out/sw4_$tag.log 2>&1 && echo "$tag $(grep '"metric"' gpurun_out/sw4_$tag.log)" >> $O || { echo "FAILED $tag" >> $O; tail -3 gpurun_out/sw4_$tag.log >> $O; }; tail -1 $O | cut -c1-200; }
b resnet50_topk
b resnet50_none --workload resnet50_none --grace-split off
b resnet50_dgc --workload resnet50_dgc
b resnet50_threshold --workload resnet50_threshold
b ddp --surface ddp --grace-split off --warmup 12
b vgg16_powersgd --workload vgg16_powersgd --steps 20
b vgg16_none --workload vgg16_none --steps 20 --grace-split off
b lstm_efsignsgd --workload lstm_efsignsgd --steps 40
b lstm_none --workload lstm_none --steps 40 --grace-split off
b bert_qsgd --workload bert_qsgd --steps 20
b bert_none --workload bert_none --steps 20 --grace-split off
b resnet18_cifar_none --workload resnet18_cifar_none --grace-split off
b resnet9_dawn --workload resnet9_dawn --grace-split off
b bf16_topk --dtype bf16 --grace-split off
