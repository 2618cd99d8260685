#!/bin/bash
# Round 3 final evidence: headline bench lines (fp32 with the grace split, bf16, uncompressed, DGC,
# Threshold), the exchange microbenchmarks, and the graphed headline kernel trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
O=gpurun_out/r3_final.txt; : > $O
b() { local tag=$1; shift; timeout -k 10 400 python bench.py --steps 30 --warmup 10 "$@" > gpurun_out/fin_$tag.log 2>&1 && python3 tools/diag/benchline.py gpurun_out/fin_$tag.log $tag >> $O || echo "FAILED $tag" >> $O; tail -1 $O; }
b headline
b headline_b
b bf16 --dtype bf16 --grace-split off
b none --workload resnet50_none --grace-split off
b dgc --workload resnet50_dgc
b threshold --workload resnet50_threshold
for p in topk dgc powersgd; do
  timeout -k 10 200 python benchmarks/grace_kernels.py --pipeline $p --iters 20 --bucket-mb 128 2>/dev/null | tail -1 >> $O || echo "grace_kernels $p failed" >> $O
done
tail -3 $O
bash tools/gpu/r3_graph_prof.sh r3final > /dev/null 2>&1; head -3 gpurun_out/prof_r3final_steps.txt
