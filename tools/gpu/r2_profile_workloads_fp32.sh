#!/bin/bash
# fp32 per-step kernel tables of the secondary BASELINE workloads (BERT QSGD, VGG-16 PowerSGD, LSTM EF-SignSGD).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
for W in bert_qsgd vgg16_powersgd lstm_efsignsgd; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof_$W" -o run -- \
    python3 "$R/bench.py" --workload $W --steps 6 --warmup 3 --exposed-steps 0 --graph off > "$R/gpurun_out/prof_$W.log" 2>&1 || exit 1
  cd "$R" && python3 tools/prof_summary.py gpurun_out/prof_$W/run_kernel_trace.csv --steps 4 --marker nll_loss_forward \
    --per-step-markers 1 --top 30 > gpurun_out/prof_${W}_steps.txt || exit 1
  rm -f gpurun_out/prof_$W/run_kernel_trace.csv; head -24 gpurun_out/prof_${W}_steps.txt
done
