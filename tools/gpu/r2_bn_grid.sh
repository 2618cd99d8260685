#!/bin/bash
# fp32 headline step: per-(kernel, grid) durations of the fused BN kernels (which layer costs
# what against its traffic), 8 eager steps under the kernel tracer.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=${1:-bn}; shift
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof_$TAG" -o run -- \
  python3 "$R/bench.py" --steps 10 --warmup 3 --exposed-steps 0 --graph off "$@" > "$R/gpurun_out/prof_$TAG.log" 2>&1 || exit 1
cd "$R" && python3 tools/prof_summary.py gpurun_out/prof_$TAG/run_kernel_trace.csv --steps 8 --marker nll_loss_forward \
  --per-step-markers 1 --top 50 > gpurun_out/prof_${TAG}_steps.txt &&
python3 tools/trace_by_grid.py gpurun_out/prof_$TAG/run_kernel_trace.csv --match grace::bn_ --top 80 > gpurun_out/prof_${TAG}_bngrid.txt &&
python3 tools/trace_seq.py gpurun_out/prof_$TAG/run_kernel_trace.csv --match grace::bn_ > gpurun_out/prof_${TAG}_bnseq.txt &&
python3 tools/trace_seq.py gpurun_out/prof_$TAG/run_kernel_trace.csv > gpurun_out/prof_${TAG}_allseq.txt &&
python3 tools/trace_by_grid.py gpurun_out/prof_$TAG/run_kernel_trace.csv --match SubTensorOp --top 40 > gpurun_out/prof_${TAG}_fillgrid.txt
rm -f gpurun_out/prof_$TAG/run_kernel_trace.csv; head -30 gpurun_out/prof_${TAG}_steps.txt
