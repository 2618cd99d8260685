#!/bin/bash
# Round 5 sweep: every BASELINE config (compressed + uncompressed), fp32, one GPU.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; mkdir -p gpurun_out
O=gpurun_out/r5_sweep_b.txt; : > $O
b() { local tag=$1; shift; timeout -k 10 400 python bench.py --steps 30 --warmup 10 "$@" > gpurun_out/sw5_$tag.log 2>&1 && echo "$tag $(grep '"metric"' gpurun_out/sw5_$tag.log)" >> $O || { echo "FAILED $tag" >> $O; tail -3 gpurun_out/sw5_$tag.log >> $O; exit 1; }; tail -1 $O | cut -c1-140; }
b lstm_efsignsgd --workload lstm_efsignsgd --steps 40
b lstm_none --workload lstm_none --steps 40
b bert_qsgd --workload bert_qsgd --steps 20
b bert_none --workload bert_none --steps 20
b resnet9_dawn --workload resnet9_dawn
b resnet18_cifar_none --workload resnet18_cifar_none
b resnet50_topk_bf16 --dtype bf16
b resnet50_topk_ddp --surface ddp
