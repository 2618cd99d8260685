#!/bin/bash
# fp32 BN parity tests + fp32 headline bench + kernel trace of the fp32 step.
#   gpurun --timeout 900 -- 'bash tools/gpu/r2_fp32.sh [extra bench args]'
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bnact.py -x -q --timeout 120 --timeout-method thread > gpurun_out/bntests.log 2>&1; rc=$?
tail -3 gpurun_out/bntests.log; [ $rc -eq 0 ] || exit $rc
printf -- "%s\n" "--steps 30 --warmup 10 $*" "--workload resnet50_none --steps 30 --warmup 10 $*" > gpurun_out/sweep_fp32.txt
bash tools/bench_sweep.sh gpurun_out/sweep_fp32.txt || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof" -o run -- \
  python3 "$R/bench.py" --steps 10 --warmup 5 --exposed-steps 0 "$@" > "$R/gpurun_out/prof.log" 2>&1 || exit 1
cd "$R" && python3 tools/prof_summary.py gpurun_out/prof/run_kernel_trace.csv --steps 8 --marker sgd_kernel \
  --per-step-markers 1 --top 45 > gpurun_out/prof_summary.txt; rm -f gpurun_out/prof/run_kernel_trace.csv; head -60 gpurun_out/prof_summary.txt
