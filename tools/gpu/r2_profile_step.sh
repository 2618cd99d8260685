#!/bin/bash
# Per-step kernel table of a bench workload (eager steps: every kernel of every step traced;
# kernel durations are the same as under the whole-step graph).  Usage: r2_profile_step.sh TAG [bench args]
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=$1; shift
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$TAG" -o run -- \
  python3 "$R/bench.py" --steps 10 --warmup 2 --exposed-steps 0 --graph off "$@" > "$R/gpurun_out/prof_$TAG.log" 2>&1 || exit 1
cd "$R" && python3 tools/prof_stats.py gpurun_out/prof_$TAG/run_kernel_stats.csv --top 40 --per 12 > gpurun_out/prof_${TAG}_stats.txt
rm -f gpurun_out/prof_$TAG/run_kernel_trace.csv; head -45 gpurun_out/prof_${TAG}_stats.txt
