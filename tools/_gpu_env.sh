# A/B of MIOpen solver/find-mode environment settings on the headline bench (one process each)
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
run() { echo "== $*"; env "$@" timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/env_last.log 2>&1 || { tail -3 gpurun_out/env_last.log; return 1; }; grep '"metric"' gpurun_out/env_last.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"; }
run A=1 &&
run MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 &&
run MIOPEN_FIND_MODE=1 &&
run MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 &&
run MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_FWD_GTC_XDLOPS_NHWC=0
