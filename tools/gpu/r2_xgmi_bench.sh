#!/bin/bash
# The one-shot xGMI all-gather inside the whole-step graph of the real bench (W = 1 through the
# RCCL process group: the pull kernels run, no peers) next to the native-inline RCCL comm.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python bench.py --force-dist --comm xgmi --steps 30 --warmup 10 > gpurun_out/bench_xgmi.log 2>&1 &&
grep '"metric"' gpurun_out/bench_xgmi.log > gpurun_out/bench_xgmi.json && cut -c1-160 gpurun_out/bench_xgmi.json &&
grep -o '"comm": "[^"]*"' gpurun_out/bench_xgmi.json &&
timeout -k 10 300 python bench.py --force-dist --comm native-inline --steps 30 --warmup 10 > gpurun_out/bench_ninl.log 2>&1 &&
grep '"metric"' gpurun_out/bench_ninl.log | cut -c1-160
