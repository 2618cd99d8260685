#!/bin/bash
# Round 4: secondary lines on the final code -- bf16 headline and the DDP comm-hook surface.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; mkdir -p gpurun_out
O=gpurun_out/r4_sec.txt; : > $O
b() { local tag=$1; shift; timeout -k 10 400 python bench.py --steps 30 --warmup 12 "$@" > gpurun_out/sec_$tag.log 2>&1 && echo "$tag $(grep '"metric"' gpurun_out/sec_$tag.log)" >> $O || { echo "FAILED $tag" >> $O; tail -3 gpurun_out/sec_$tag.log >> $O; exit 1; }; tail -1 $O | cut -c1-160; }
b bf16_topk --dtype bf16
b ddp --surface ddp --bf16-weights off
b engine
# MIOpen's GTC NHWC bwd/wrw solvers zero their output first (SubTensorOpWithScalar1d, 70 launches/step):
# A/B against letting MIOpen find pick among the other solvers.
MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 b no_gtc_wrw
MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 b no_gtc_bwd
