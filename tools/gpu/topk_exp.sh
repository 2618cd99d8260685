#!/bin/bash
# Top-K split-kernel experiment: kernel times with parts of the work disabled (GRACE_TOPK_DBG bits:
# 1 = no slot atomics, 2 = no output writes, 4 = no candidate histogram atomics).  Timing only.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
for D in 0 1 3 4 7; do
  cd /tmp && GRACE_TOPK_DBG=$D timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/texp$D" -o run -- \
    python3 "$R/benchmarks/grace_kernels.py" --pipeline topk --iters 20 --no-graph "$@" > /dev/null 2>&1 || exit 1
  cd "$R" && echo "== dbg $D" && python3 tools/prof_stats.py gpurun_out/texp$D/run_kernel_stats.csv --top 12 --per 23 | grep -i "topk\|total"
  rm -f gpurun_out/texp$D/run_kernel_trace.csv
done
