#!/bin/bash
# rocprofv3 kernel trace of one bench.py configuration -> per-step kernel table + per-queue view.
#   gpurun --timeout 600 -- 'bash tools/gpu/profile.sh TAG [bench.py args]'
# Summaries: gpurun_out/prof_TAG_summary.txt (copy the ones to keep to profiles/)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=$1; shift
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof_$TAG" -o run -- \
  python3 "$R/bench.py" --steps 10 --warmup 5 --grace-split off --exposed-steps 0 "$@" > "$R/gpurun_out/prof_$TAG.log" 2>&1 || exit 1
cd "$R" && CSV=gpurun_out/prof_$TAG/run_kernel_trace.csv &&
{ tail -1 gpurun_out/prof_$TAG.log; python3 tools/prof_summary.py $CSV --steps 8 --marker nll_loss_forward --per-step-markers 1 --top 40;
  python3 tools/trace_streams.py $CSV --steps 8 --marker nll_loss_forward --tail 40;
  python3 tools/trace_gaps.py $CSV --steps 4 --marker nll_loss_forward --top 30; } > gpurun_out/prof_${TAG}_summary.txt 2>&1
rc=$?; gzip -f $CSV; head -30 gpurun_out/prof_${TAG}_summary.txt; exit $rc
