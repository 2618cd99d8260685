#!/bin/bash
# Round 3: kernel trace of the GRAPHED fp32 headline step (wgrad side stream on): busy time,
# idle gaps, per-kernel table; then bench A/B of the GRACE exchange overlap / bucket size.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=${1:-r3g}
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof_$TAG" -o run -- \
  python3 "$R/bench.py" --steps 10 --warmup 6 --exposed-steps 0 --grace-split off > "$R/gpurun_out/prof_$TAG.log" 2>&1 || exit 1
cd "$R" && python3 tools/prof_summary.py gpurun_out/prof_$TAG/run_kernel_trace.csv --steps 8 --marker nll_loss_forward \
  --per-step-markers 1 --top 60 --gaps 25 > gpurun_out/prof_${TAG}_steps.txt &&
python3 tools/trace_seq.py gpurun_out/prof_$TAG/run_kernel_trace.csv > gpurun_out/prof_${TAG}_allseq.txt || exit 1
rm -f gpurun_out/prof_$TAG/run_kernel_trace.csv; head -40 gpurun_out/prof_${TAG}_steps.txt
B='"value": [0-9.]*, "unit": "images/s", "n_gpus": 1, "steps": 30, "warmup": 10, "ms_per_step": [0-9.]*'
run() { local tag=$1; shift; echo "$tag:"; timeout -k 10 300 python bench.py --steps 30 --warmup 10 --grace-split off --exposed-steps 0 "$@" > gpurun_out/r3_ov_$tag.log 2>&1 && grep -o "$B" gpurun_out/r3_ov_$tag.log; }
run base &&
run ov128 --overlap on &&
run ov32 --overlap on --bucket-mb 32 &&
run ov16 --overlap on --bucket-mb 16 &&
run base_b
