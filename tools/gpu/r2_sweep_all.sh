#!/bin/bash
# Every BASELINE workload at fp32 (the reference precision) + the uncompressed point (part 1),
# then the bf16 secondary runs, stock-PyTorch reference points and the W=2 gloo rehearsal
# (part 2).  One process each, 1 GPU.   usage: r2_sweep_all.sh 1|2
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
if [ "${1:-1}" = 1 ]; then
printf -- "%s\n" "--steps 30 --warmup 10" "--workload resnet50_none --steps 30 --warmup 10" \
  "--workload vgg16_powersgd --steps 20 --warmup 10" "--workload vgg16_none --steps 20 --warmup 10" \
  "--workload lstm_efsignsgd --steps 40 --warmup 10" "--workload lstm_none --steps 40 --warmup 10" \
  "--workload bert_qsgd --steps 20 --warmup 10" "--workload bert_none --steps 20 --warmup 10" \
  "--workload resnet50_dgc --steps 30 --warmup 10" \
  "--workload resnet9_dawn --steps 30 --warmup 10" "--workload resnet18_cifar_none --steps 30 --warmup 10" \
  > gpurun_out/sweep_p1.txt
bash tools/bench_sweep.sh gpurun_out/sweep_p1.txt | tee gpurun_out/sweep_p1.out
else
printf -- "%s\n" "--dtype bf16 --steps 30 --warmup 10" "--workload resnet50_none --dtype bf16 --steps 30 --warmup 10" \
  "--workload vgg16_powersgd --dtype bf16 --steps 20 --warmup 10" \
  "--workload lstm_efsignsgd --dtype bf16 --steps 40 --warmup 10" "--workload bert_qsgd --dtype bf16 --steps 20 --warmup 10" \
  "GRACE_AMD_FORCE_TORCH=1 --workload resnet50_none --optimizer torch --steps 30 --warmup 10" \
  "GRACE_AMD_FORCE_TORCH=1 --workload resnet50_none --optimizer torch --graph off --steps 30 --warmup 10" \
  > gpurun_out/sweep_p2.txt
bash tools/bench_sweep.sh gpurun_out/sweep_p2.txt | tee gpurun_out/sweep_p2.out || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 \
  bench.py --gpus 2 --backend gloo --steps 10 --warmup 5 > gpurun_out/w2_gloo.log 2>&1 && grep '"metric"' gpurun_out/w2_gloo.log | cut -c1-400
fi
