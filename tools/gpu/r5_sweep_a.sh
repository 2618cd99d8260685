#!/bin/bash
# Round 5 sweep: every BASELINE config (compressed + uncompressed), fp32, one GPU.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; mkdir -p gpurun_out
O=gpurun_out/r5_sweep_a.txt; : > $O
b() { local tag=$1; shift; timeout -k 10 400 python bench.py --steps 30 --warmup 10 "$@" > gpurun_out/sw5_$tag.log 2>&1 && echo "$tag $(grep '"metric"' gpurun_out/sw5_$tag.log)" >> $O || { echo "FAILED $tag" >> $O; tail -3 gpurun_out/sw5_$tag.log >> $O; exit 1; }; tail -1 $O | cut -c1-140; }
b resnet50_topk
b resnet50_none --workload resnet50_none
b resnet50_dgc --workload resnet50_dgc
b resnet50_threshold --workload resnet50_threshold
b vgg16_powersgd --workload vgg16_powersgd --steps 20
b vgg16_none --workload vgg16_none --steps 20
