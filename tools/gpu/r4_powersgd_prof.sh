#!/bin/bash
# Round 4: PowerSGD exchange (VGG-16 gradients) kernel profile.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; mkdir -p gpurun_out
timeout -k 10 200 python benchmarks/grace_kernels.py --pipeline powersgd > gpurun_out/r4_ps_bench.txt 2>&1 || { tail -20 gpurun_out/r4_ps_bench.txt; exit 1; }
cat gpurun_out/r4_ps_bench.txt | tail -5
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_ps" -o run -- python3 "$R/benchmarks/grace_kernels.py" --pipeline powersgd --no-graph > "$R/gpurun_out/prof_ps.log" 2>&1 || { tail -5 "$R/gpurun_out/prof_ps.log"; exit 1; }
cd "$R" && head -30 gpurun_out/prof_ps/run_kernel_stats.csv | cut -d, -f1-8
