#!/bin/bash
# capacity-payload codecs: GPU tests (graph replay == eager), DGC workload bench with the whole-step graph
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_capacity_graph.py tests/test_gpu_compressors.py tests/test_gpu_multirank.py -x -q --timeout 200 --timeout-method thread > gpurun_out/captests.log 2>&1; rc=$?
tail -5 gpurun_out/captests.log; [ $rc -eq 0 ] || exit $rc
printf -- "%s\n" "--workload resnet50_dgc --steps 30 --warmup 10" "--workload resnet50_dgc --steps 30 --warmup 10 --graph off" > gpurun_out/sweep_dgc.txt
bash tools/bench_sweep.sh gpurun_out/sweep_dgc.txt
