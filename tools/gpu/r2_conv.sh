#!/bin/bash
# fp32 per-layer conv timing (MIOpen channels-last / NCHW / 1x1-as-GEMM) + the fp32 headline's
# per-step kernel table.   gpurun --timeout 900 -- 'bash tools/gpu/r2_conv.sh'
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 420 python -u benchmarks/conv_bench.py "$@" > gpurun_out/conv_bench.txt 2>&1 || { tail -20 gpurun_out/conv_bench.txt; exit 1; }
tail -8 gpurun_out/conv_bench.txt
bash tools/gpu/r2_profile_step.sh r50fp32
