#!/bin/bash
# Sketch native select: GPU tests + exchange microbench, then the fp32 sweep of every BASELINE workload.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sketch.py -x -v --timeout 120 --timeout-method thread > gpurun_out/sktests.log 2>&1; rc=$?
tail -8 gpurun_out/sktests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python benchmarks/grace_kernels.py --pipeline sketch,topk > gpurun_out/gk_sketch.log 2>&1 || { tail gpurun_out/gk_sketch.log; exit 1; }
grep -v amdgpu.ids gpurun_out/gk_sketch.log
[ "$1" = "nosweep" ] && exit 0
printf -- "%s\n" "--workload vgg16_powersgd --steps 20 --warmup 10" "--workload vgg16_none --steps 20 --warmup 10" \
  "--workload lstm_efsignsgd --steps 40 --warmup 10" "--workload lstm_none --steps 40 --warmup 10" \
  "--workload bert_qsgd --steps 20 --warmup 10" "--workload bert_none --steps 20 --warmup 10" \
  "--workload resnet50_none --steps 30 --warmup 10" "--steps 30 --warmup 10" > gpurun_out/sweep_fp32_all.txt
bash tools/bench_sweep.sh gpurun_out/sweep_fp32_all.txt | tee gpurun_out/sweep_fp32_all.out
