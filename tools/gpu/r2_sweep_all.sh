#!/bin/bash
# Every BASELINE workload at fp32 (the reference precision) + the uncompressed point, then the
# compressed ones at bf16 (secondary).  One process each, 1 GPU.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
printf -- "%s\n" "--steps 30 --warmup 10" "--workload resnet50_none --steps 30 --warmup 10" \
  "--workload vgg16_powersgd --steps 20 --warmup 10" "--workload vgg16_none --steps 20 --warmup 10" \
  "--workload lstm_efsignsgd --steps 40 --warmup 10" "--workload lstm_none --steps 40 --warmup 10" \
  "--workload bert_qsgd --steps 20 --warmup 10" "--workload bert_none --steps 20 --warmup 10" \
  "--workload resnet50_dgc --steps 30 --warmup 10" \
  "--workload resnet9_dawn --steps 30 --warmup 10" "--workload resnet18_cifar_none --steps 30 --warmup 10" \
  "--dtype bf16 --steps 30 --warmup 10" "--workload vgg16_powersgd --dtype bf16 --steps 20 --warmup 10" \
  "--workload lstm_efsignsgd --dtype bf16 --steps 40 --warmup 10" "--workload bert_qsgd --dtype bf16 --steps 20 --warmup 10" \
  "GRACE_AMD_FORCE_TORCH=1 --workload resnet50_none --optimizer torch --steps 30 --warmup 10" \
  "GRACE_AMD_FORCE_TORCH=1 --workload resnet50_none --optimizer torch --graph off --steps 30 --warmup 10" \
  > gpurun_out/sweep_all_r2.txt
bash tools/bench_sweep.sh gpurun_out/sweep_all_r2.txt
