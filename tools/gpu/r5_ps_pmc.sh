#!/bin/bash
# PMC counters of the PowerSGD exchange kernels (VGG-16, 128 MB buckets): occupancy, waits, bytes.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=$R/gpurun_out/pspmc; mkdir -p $D
cd /tmp
P="python3 $R/benchmarks/grace_kernels.py --pipeline powersgd --iters 2 --no-graph --bucket-mb 128"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU \
  --output-format csv -d $D/a -o run -- $P > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/b -o run -- $P > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/c -o run -- $P > /dev/null 2>&1 || exit 1
cd $R && python3 tools/pmc_summary.py $(find $D/a $D/b $D/c -name '*counter_collection.csv') --grace --top 12 | cut -c1-300
