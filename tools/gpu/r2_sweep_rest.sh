#!/bin/bash
# remaining fp32 workloads + the bf16 secondary runs (one process each, 1 GPU)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
printf -- "%s\n" "--workload resnet50_dgc --steps 30 --warmup 10" \
  "--workload resnet9_dawn --steps 30 --warmup 10" "--workload resnet18_cifar_none --steps 30 --warmup 10" \
  "--dtype bf16 --steps 30 --warmup 10" "--workload resnet50_none --dtype bf16 --steps 30 --warmup 10" \
  "--workload vgg16_powersgd --dtype bf16 --steps 20 --warmup 10" \
  "--workload lstm_efsignsgd --dtype bf16 --steps 40 --warmup 10" "--workload bert_qsgd --dtype bf16 --steps 20 --warmup 10" \
  "--workload resnet9_dawn --dtype bf16 --steps 30 --warmup 10" > gpurun_out/sweep_rest.txt
bash tools/bench_sweep.sh gpurun_out/sweep_rest.txt | tee gpurun_out/sweep_rest.out
