#!/bin/bash
# Round 4: ADVICE fixes on the GPU (wgrad joinable rule, xGMI slot publish + probe, health words,
# overflow counter), W=2 whole-step-graph rehearsal (gloo bootstrap, xGMI one-shot exchange).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_a_comm.py tests/test_gpu_wgrad.py \
  tests/test_gpu_xgmi.py tests/test_gpu_capacity_graph.py tests/test_gpu_engine.py > gpurun_out/r4_check1_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r4_check1_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/r4_bench1.log 2>&1 || { echo bench failed; tail -5 gpurun_out/r4_bench1.log; exit 1; }
tail -1 gpurun_out/r4_bench1.log | cut -c1-400; grep -c "AccumulateGrad" gpurun_out/r4_bench1.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 \
  bench.py --gpus 2 --backend gloo --comm auto --graph full --steps 20 --warmup 6 > gpurun_out/r4_w2_rehearsal.log 2>&1 || { echo w2 failed; tail -20 gpurun_out/r4_w2_rehearsal.log; exit 1; }
grep '"metric"' gpurun_out/r4_w2_rehearsal.log | cut -c1-1500
