#!/bin/bash
# Graphed headline kernel tables: default vs GRACE_BN_PROLOGUE=2 (bn2 apply inside conv3's GEMM).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=$R/gpurun_out/proprof; mkdir -p $D
for m in 0 2; do
  cd /tmp && GRACE_BN_PROLOGUE=$m timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/p$m -o run -- \
    python3 $R/bench.py --steps 10 --warmup 5 > $D/p$m.log 2>&1 || exit 1
  cd $R && python3 tools/prof_summary.py $D/p$m/run_kernel_trace.csv --steps 8 --marker topk2_split --per-step-markers 1 \
    --top 40 > $D/sum$m.txt && rm -f $D/p$m/run_kernel_trace.csv && head -30 $D/sum$m.txt | cut -c1-150 || exit 1
done
