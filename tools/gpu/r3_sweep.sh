#!/bin/bash
# Round 3 evidence sweep: GRACE exchange microbenchmarks (one 128 MB bucket), then bench lines for
# the headline (with the graphed grace_ms split), DGC, Threshold (bytes on the wire), the DDP
# comm-hook surface, bf16, and the uncompressed reference.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
O=gpurun_out/r3_sweep.txt; : > $O
for p in topk powersgd sketch dgc threshold qsgd efsignsgd; do
  timeout -k 10 200 python benchmarks/grace_kernels.py --pipeline $p --iters 20 --bucket-mb 128 2>/dev/null | tail -1 >> $O || { echo "grace_kernels $p failed" >> $O; }
done
cat $O
b() { local tag=$1; shift; echo "== $tag" >> $O; timeout -k 10 400 python bench.py --steps 30 --warmup 10 "$@" > gpurun_out/sw_$tag.log 2>&1 && grep '"metric"' gpurun_out/sw_$tag.log >> $O || { echo "FAILED $tag" >> $O; tail -3 gpurun_out/sw_$tag.log >> $O; }; tail -1 $O | cut -c1-400; }
b headline
b none --workload resnet50_none --grace-split off
b dgc --workload resnet50_dgc
b threshold --workload resnet50_threshold
b ddp --surface ddp --grace-split off
b bf16 --dtype bf16 --grace-split off
