#!/bin/bash
# fp32 headline with MIOpen's asm GTC implicit-GEMM solvers (which zero their outputs with
# SubTensorOp memsets) disabled per direction: does find pick a faster total without them?
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
run() { echo "== $1"; shift; env "$@" timeout -k 10 300 python bench.py --steps 30 --warmup 10 --exposed-steps 0 > gpurun_out/mexp.log 2>&1 || { tail -3 gpurun_out/mexp.log; return 1; }
  grep '"metric"' gpurun_out/mexp.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"; }
run default A=1 &&
run no_wrw_gtc MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 &&
run no_bwd_gtc MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 &&
run no_fwd_gtc MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_FWD_GTC_XDLOPS_NHWC=0 &&
run no_gtc_all MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_FWD_GTC_XDLOPS_NHWC=0
