#!/bin/bash
# Headline bench under MIOpen solver restrictions (the ASM implicit-GEMM wrw/bwd solvers need
# fp32 workspace zeroing + cast kernels around every call) + an RCCL-in-graph check
# (--force-dist) + a kernel-neighbour trace of the library memsets.
#   gpurun --timeout 900 -- 'bash tools/gpu/miopen_sweep.sh'
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
B="python bench.py --steps 30 --warmup 10"
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 240 $B > gpurun_out/sweep_$name.log 2>&1 || { tail -5 gpurun_out/sweep_$name.log; exit 1; }
  echo "$name $(tail -1 gpurun_out/sweep_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["hip_graph"])')"
}
run base X=1
run nowrw MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0
run nobwd MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0
run noasm MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0
env timeout -k 10 240 $B --force-dist > gpurun_out/sweep_forcedist.log 2>&1 || { tail -5 gpurun_out/sweep_forcedist.log; exit 1; }
echo "forcedist $(tail -1 gpurun_out/sweep_forcedist.log)"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof" -o run -- \
  python3 "$R/bench.py" --steps 10 --warmup 5 > "$R/gpurun_out/prof.log" 2>&1 || exit 1
cd "$R" && python3 tools/trace_neighbors.py gpurun_out/prof/run_kernel_trace.csv --last 3000 \
  --match fillBufferAligned --match SubTensorOpWithScalar1d --match SubTensorOpWithCastTensor1d \
  --match multi_tensor_apply --match CUDAFunctor_add --match bfloat16tofloat32 > gpurun_out/neighbors.txt &&
python3 tools/prof_summary.py gpurun_out/prof/run_kernel_trace.csv --steps 8 --marker Cijk_Alik_Bljk \
  --per-step-markers 1 --top 45 > gpurun_out/prof_summary.txt && gzip -f gpurun_out/prof/run_kernel_trace.csv &&
cat gpurun_out/neighbors.txt
