#!/bin/bash
# Round 3: kernel trace of the fp32 headline step (eager steps under rocprofv3 --kernel-trace; the
# conv autotune runs in the warmup steps) -> per-step kernel table + full kernel sequence.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=${1:-r3}; shift
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof_$TAG" -o run -- \
  python3 "$R/bench.py" --steps 10 --warmup 3 --exposed-steps 0 --graph off --grace-split off "$@" > "$R/gpurun_out/prof_$TAG.log" 2>&1 || exit 1
cd "$R" && python3 tools/prof_summary.py gpurun_out/prof_$TAG/run_kernel_trace.csv --steps 8 --marker nll_loss_forward \
  --per-step-markers 1 --top 70 > gpurun_out/prof_${TAG}_steps.txt &&
python3 tools/trace_seq.py gpurun_out/prof_$TAG/run_kernel_trace.csv > gpurun_out/prof_${TAG}_allseq.txt &&
python3 tools/trace_by_grid.py gpurun_out/prof_$TAG/run_kernel_trace.csv --match SubTensorOp --top 40 > gpurun_out/prof_${TAG}_fillgrid.txt
rm -f gpurun_out/prof_$TAG/run_kernel_trace.csv; head -75 gpurun_out/prof_${TAG}_steps.txt
