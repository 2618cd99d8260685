#!/bin/bash
# Per-step kernel table of a bench workload over the last 8 eager steps (every kernel traced;
# durations as under the whole-step graph; MIOpen find happens in the warm-up steps and is
# outside the window).  Usage: r2_profile_step.sh TAG [bench args]
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=$1; shift
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof_$TAG" -o run -- \
  python3 "$R/bench.py" --steps 10 --warmup 3 --exposed-steps 0 --graph off "$@" > "$R/gpurun_out/prof_$TAG.log" 2>&1 || exit 1
cd "$R" && python3 tools/prof_summary.py gpurun_out/prof_$TAG/run_kernel_trace.csv --steps 8 --marker nll_loss_forward \
  --per-step-markers 1 --top 50 > gpurun_out/prof_${TAG}_steps.txt
rm -f gpurun_out/prof_$TAG/run_kernel_trace.csv; head -56 gpurun_out/prof_${TAG}_steps.txt
