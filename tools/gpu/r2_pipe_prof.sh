#!/bin/bash
# Exchange microbenchmark of one pipeline: graph-replayed time + per-kernel stats (+PMC optional)
# usage: r2_pipe_prof.sh PIPELINE [--pmc]
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
P=$1
timeout -k 10 200 python benchmarks/grace_kernels.py --pipeline $P --iters 30 > gpurun_out/gk_$P.log 2>&1 || { tail -5 gpurun_out/gk_$P.log; exit 1; }
tail -1 gpurun_out/gk_$P.log
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$P" -o run -- \
  python3 "$R/benchmarks/grace_kernels.py" --pipeline $P --iters 20 --no-graph > /dev/null 2>&1 || exit 1
cd "$R" && python3 tools/prof_stats.py gpurun_out/prof_$P/run_kernel_stats.csv --top 20 --per 23 > gpurun_out/prof_${P}_stats.txt; cat gpurun_out/prof_${P}_stats.txt
python3 tools/trace_by_grid.py gpurun_out/prof_$P/run_kernel_trace.csv --match grace --top 30 > gpurun_out/prof_${P}_grid.txt; cat gpurun_out/prof_${P}_grid.txt
rm -f gpurun_out/prof_$P/run_kernel_trace.csv
if [ "$2" == "--pmc" ]; then
  cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES \
    --output-format csv -d "$R/gpurun_out/pmc_${P}_a" -o run -- python3 "$R/benchmarks/grace_kernels.py" --pipeline $P --iters 2 --no-graph > /dev/null 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_${P}_b" -o run -- \
    python3 "$R/benchmarks/grace_kernels.py" --pipeline $P --iters 2 --no-graph > /dev/null 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_${P}_c" -o run -- \
    python3 "$R/benchmarks/grace_kernels.py" --pipeline $P --iters 2 --no-graph > /dev/null 2>&1 || exit 1
  cd "$R" && python3 tools/pmc_summary.py $(find gpurun_out/pmc_${P}_? -name '*counter_collection.csv') --grace > gpurun_out/pmc_${P}_summary.txt && cat gpurun_out/pmc_${P}_summary.txt
fi
