#!/bin/bash
# Round 4: per-shape fp32 BN kernel times (graph-replayed) under grid / reduction knobs.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
O=gpurun_out/r4_bnbench.txt; : > $O
for cfg in "base" "GRACE_BN_ATOMIC_CHUNKS=0" "GRACE_BN_TARGET_BLOCKS=1024" "GRACE_BN_VPT_MIN=4"; do
  echo "== $cfg" >> $O
  if [ "$cfg" = base ]; then e=""; else e="$cfg"; fi
  env $e timeout -k 10 200 python benchmarks/bnact_bench.py --dtype fp32 --iters 20 >> $O 2>&1 || { echo "FAILED $cfg" >> $O; break; }
done
cat $O
