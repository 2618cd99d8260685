#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_compressors.py tests/test_gpu_multirank.py tests/test_gpu_graph_rng.py -x -q -k "powersgd or multirank or graph or rng" --timeout 200 --timeout-method thread > gpurun_out/pstests.log 2>&1; rc=$?
tail -3 gpurun_out/pstests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/r2_pipe_prof.sh powersgd && timeout -k 10 300 python bench.py --workload vgg16_powersgd --steps 20 --warmup 10 > gpurun_out/bench_vgg.log 2>&1; grep '"metric"' gpurun_out/bench_vgg.log | cut -c1-400
