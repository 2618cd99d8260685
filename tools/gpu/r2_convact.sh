#!/bin/bash
# Fused conv bias+ReLU: GPU tests, VGG-16 PowerSGD fp32 bench (before: 1103 img/s, 29.00 ms), kernel table.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_convact.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/convact_tests.log 2>&1; rc=$?; tail -2 gpurun_out/convact_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --workload vgg16_powersgd --steps 20 --warmup 10 > gpurun_out/bench_vgg.log 2>&1 && tail -1 gpurun_out/bench_vgg.log | cut -c1-220 &&
timeout -k 10 400 python bench.py --workload vgg16_none --steps 20 --warmup 10 > gpurun_out/bench_vgg_none.log 2>&1 && tail -1 gpurun_out/bench_vgg_none.log | cut -c1-220 &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof_vggca" -o run -- \
    python3 "$R/bench.py" --workload vgg16_powersgd --steps 6 --warmup 3 --exposed-steps 0 --graph off > "$R/gpurun_out/prof_vggca.log" 2>&1 &&
cd "$R" && python3 tools/prof_summary.py gpurun_out/prof_vggca/run_kernel_trace.csv --steps 4 --marker nll_loss_forward \
    --per-step-markers 1 --top 30 > gpurun_out/prof_vggca_steps.txt && rm -f gpurun_out/prof_vggca/run_kernel_trace.csv && head -26 gpurun_out/prof_vggca_steps.txt
