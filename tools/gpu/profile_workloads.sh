#!/bin/bash
# rocprofv3 kernel tables of the BERT QSGD and VGG-16 PowerSGD benches (per-step window on the SGD kernel).
R=${GRAFT_REPO_ROOT}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
for W in bert_qsgd vgg16_powersgd; do
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof_$W" -o run -- python3 "$R/bench.py" --workload $W --steps 8 --warmup 4 > "$R/gpurun_out/prof_$W.log" 2>&1 || exit 1
cd "$R" && python3 tools/prof_summary.py gpurun_out/prof_$W/run_kernel_trace.csv --steps 6 --marker sgd_kernel --per-step-markers 0 --top 30 > gpurun_out/prof_${W}_summary.txt 2>&1; python3 tools/trace_by_grid.py gpurun_out/prof_$W/run_kernel_trace.csv --match grace --top 25 >> gpurun_out/prof_${W}_summary.txt; rm -f gpurun_out/prof_$W/run_kernel_trace.csv; cat gpurun_out/prof_${W}_summary.txt
done
