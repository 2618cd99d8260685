#!/bin/bash
# native comm group tests + a W=2 bench.py rehearsal (2 gloo ranks sharing the GPU) + W=1 RCCL path
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_a_comm.py -x -q --timeout 200 --timeout-method thread > gpurun_out/commtests.log 2>&1; rc=$?
tail -3 gpurun_out/commtests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 \
  bench.py --gpus 2 --steps 20 --warmup 5 --backend gloo > gpurun_out/bench_w2_gloo.log 2>&1; rc=$?
grep '"metric"' gpurun_out/bench_w2_gloo.log; tail -3 gpurun_out/bench_w2_gloo.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --force-dist > gpurun_out/bench_w1_rccl.log 2>&1; rc=$?
grep '"metric"' gpurun_out/bench_w1_rccl.log; exit $rc
