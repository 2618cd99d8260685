#!/bin/bash
# Top-K numerics + exchange microbenchmark (+ optional PMC pass) + headline bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_topk.py tests/test_gpu_compressors.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/topktests.log 2>&1; rc=$?
tail -3 gpurun_out/topktests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python benchmarks/grace_kernels.py --pipeline topk --iters 50 > gpurun_out/gk_topk.log 2>&1 && timeout -k 10 200 python benchmarks/grace_kernels.py --pipeline topk --iters 50 --bucket-mb 128 >> gpurun_out/gk_topk.log 2>&1; rc=$?
tail -4 gpurun_out/gk_topk.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_topk" -o run -- \
  python3 "$R/benchmarks/grace_kernels.py" --pipeline topk --iters 20 --no-graph > /dev/null 2>&1 || exit 1
cd "$R" && python3 tools/prof_stats.py gpurun_out/prof_topk/run_kernel_stats.csv --top 20 --per 23 > gpurun_out/prof_topk_stats.txt; cat gpurun_out/prof_topk_stats.txt
rm -f gpurun_out/prof_topk/run_kernel_trace.csv
# PMC: LDS conflicts / busy of the Top-K kernels, then HBM bytes (separate passes)
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES \
  --output-format csv -d "$R/gpurun_out/pmc_topk_a" -o run -- python3 "$R/benchmarks/grace_kernels.py" --pipeline topk --iters 2 --no-graph > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_topk_b" -o run -- \
  python3 "$R/benchmarks/grace_kernels.py" --pipeline topk --iters 2 --no-graph > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_topk_c" -o run -- \
  python3 "$R/benchmarks/grace_kernels.py" --pipeline topk --iters 2 --no-graph > /dev/null 2>&1 || exit 1
cd "$R" && python3 tools/pmc_summary.py $(find gpurun_out/pmc_topk_? -name '*counter_collection.csv') --grace > gpurun_out/pmc_topk_summary.txt && cat gpurun_out/pmc_topk_summary.txt
cd "$R" && timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log; exit $rc
