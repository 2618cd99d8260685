#!/bin/bash
# rocprofv3 kernel trace of the headline bench -> per-step kernel table (+ per-grid BN/GRACE
# rows), and PMC passes (SQ cycles/MFMA/LDS conflicts, FETCH/WRITE_SIZE) over the GRACE
# exchange microbenchmark.  Summaries land in gpurun_out/ (copy the ones to keep to profiles/).
#   gpurun --timeout 900 -- 'bash tools/gpu/profile_headline.sh [extra bench.py args]'
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof" -o run -- \
  python3 "$R/bench.py" --steps 10 --warmup 5 "$@" > "$R/gpurun_out/prof.log" 2>&1 || exit 1
cd "$R" && python3 tools/prof_summary.py gpurun_out/prof/run_kernel_trace.csv --steps 8 --marker Cijk_Alik_Bljk \
  --per-step-markers 1 --top 45 > gpurun_out/prof_summary.txt &&
python3 tools/trace_by_grid.py gpurun_out/prof/run_kernel_trace.csv --match grace --top 40 >> gpurun_out/prof_summary.txt &&
rm -f gpurun_out/prof/run_kernel_trace.csv && head -50 gpurun_out/prof_summary.txt || exit 1
for P in topk powersgd; do
  cd /tmp
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT \
    SQ_LDS_IDX_ACTIVE SQ_WAVES --output-format csv -d "$R/gpurun_out/pmc_${P}_a" -o run -- \
    python3 "$R/benchmarks/grace_kernels.py" --pipeline $P --iters 2 --no-graph > /dev/null 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_${P}_b" -o run -- \
    python3 "$R/benchmarks/grace_kernels.py" --pipeline $P --iters 2 --no-graph > /dev/null 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_${P}_c" -o run -- \
    python3 "$R/benchmarks/grace_kernels.py" --pipeline $P --iters 2 --no-graph > /dev/null 2>&1 || exit 1
  cd "$R" && python3 tools/pmc_summary.py $(find gpurun_out/pmc_${P}_? -name '*counter_collection.csv') --grace \
    > gpurun_out/pmc_${P}_summary.txt || exit 1
done
