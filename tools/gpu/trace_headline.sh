#!/bin/bash
# rocprofv3 kernel trace of the headline bench only -> per-step kernel table (no PMC passes).
#   gpurun --timeout 600 -- 'bash tools/gpu/trace_headline.sh [extra bench.py args]'
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof" -o run -- \
  python3 "$R/bench.py" --steps 10 --warmup 5 "$@" > "$R/gpurun_out/prof.log" 2>&1 || exit 1
cd "$R" && python3 tools/prof_summary.py gpurun_out/prof/run_kernel_trace.csv --steps 8 --marker Cijk_Alik_Bljk \
  --per-step-markers 1 --top 60 > gpurun_out/prof_summary.txt &&
python3 tools/trace_neighbors.py gpurun_out/prof/run_kernel_trace.csv --match fillBufferAligned --match SubTensorOpWithScalar1d --last 700 \
  > gpurun_out/prof_fill_neighbors.txt 2>&1;
rm -f gpurun_out/prof/run_kernel_trace.csv; head -70 gpurun_out/prof_summary.txt
