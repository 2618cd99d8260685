#!/bin/bash
# Sketch-64 exchange kernels: SQ counters (instruction mix, LDS conflicts, LDS waits) per kernel.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
  SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d "$R/gpurun_out/pmc_sk_a" -o run -- \
  python3 "$R/benchmarks/grace_kernels.py" --pipeline sketch --iters 2 --bucket-mb 128 --no-graph > /dev/null 2>&1 || exit 1
cd "$R" && python3 tools/pmc_summary.py $(find gpurun_out/pmc_sk_a -name '*counter_collection.csv') --grace \
  > gpurun_out/pmc_sk_summary.txt && cat gpurun_out/pmc_sk_summary.txt
