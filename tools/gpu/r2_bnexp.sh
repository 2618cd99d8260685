#!/bin/bash
# fp32 per-shape BN timing + MIOpen per-direction solver exclusion on the fp32 headline.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python benchmarks/bnact_bench.py --dtype fp32 > gpurun_out/bn_fp32_shapes.txt 2>&1 || { tail gpurun_out/bn_fp32_shapes.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/bn_fp32_shapes.txt
run() { local t=$1; echo "== $t"; shift; env "$@" timeout -k 10 300 python bench.py --steps 30 --warmup 10 --exposed-steps 0 > gpurun_out/mexp_$t.log 2>&1 || { tail -3 gpurun_out/mexp_$t.log; return 1; }
  grep '"metric"' gpurun_out/mexp_$t.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"; }
[ "$1" = "nomiopen" ] && exit 0
run default A=1 &&
run no_wrw_gtc MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 &&
run no_bwd_gtc MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 &&
run no_fwd_gtc MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_FWD_GTC_XDLOPS_NHWC=0
