#!/bin/bash
# Round-2 baseline: GPU tests, smoke, headline at fp32 (reference precision) and bf16, the fp32
# uncompressed point, and a kernel trace of the fp32 headline step.
#   gpurun --timeout 1100 -- 'bash tools/gpu/r2_baseline.sh'
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1; rc=$?
tail -3 gpurun_out/gputests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log || exit 1
printf -- "%s\n" "--steps 30 --warmup 10" "--workload resnet50_none --steps 30 --warmup 10" \
  "--dtype bf16 --steps 30 --warmup 10" > gpurun_out/sweep_r2.txt
bash tools/bench_sweep.sh gpurun_out/sweep_r2.txt || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof" -o run -- \
  python3 "$R/bench.py" --steps 10 --warmup 5 > "$R/gpurun_out/prof.log" 2>&1 || exit 1
cd "$R" && python3 tools/prof_summary.py gpurun_out/prof/run_kernel_trace.csv --steps 8 --marker sgd_kernel \
  --per-step-markers 1 --top 45 > gpurun_out/prof_summary.txt; rm -f gpurun_out/prof/run_kernel_trace.csv; head -60 gpurun_out/prof_summary.txt
