#!/bin/bash
# Sketch encode finisher + packed selection histograms; DDP surface in-line wgrads + bucket views.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONUNBUFFERED=1; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_sketch.py \
  tests/test_gpu_a_comm.py > gpurun_out/skddp_tests.log 2>&1 || { tail -30 gpurun_out/skddp_tests.log; exit 1; }
tail -2 gpurun_out/skddp_tests.log
timeout -k 10 200 python benchmarks/grace_kernels.py --pipeline sketch --iters 30 --bucket-mb 128 > gpurun_out/sk_bench.log 2>&1 || exit 1
tail -2 gpurun_out/sk_bench.log
bash tools/gpu/r3_sketch_prof.sh || exit 1
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
  SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d "$R/gpurun_out/pmc_sk_a" -o run -- \
  python3 "$R/benchmarks/grace_kernels.py" --pipeline sketch --iters 2 --bucket-mb 128 --no-graph > "$R/gpurun_out/pmc_sk.log" 2>&1
echo "pmc rc $?"
cd "$R" && python3 tools/pmc_summary.py $(find gpurun_out/pmc_sk_a -name '*counter_collection.csv') --grace > gpurun_out/pmc_sk_summary.txt; cat gpurun_out/pmc_sk_summary.txt
bash tools/gpu/r3_ddp_graph.sh
