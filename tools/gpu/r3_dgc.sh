#!/bin/bash
# Round 3: DGC tree refinement -- DGC GPU tests, exchange microbench, resnet50_dgc bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_compressors.py tests/test_gpu_capacity_graph.py tests/test_gpu_graph_rng.py > gpurun_out/r3_dgc_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r3_dgc_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python benchmarks/grace_kernels.py --pipeline dgc --iters 20 --bucket-mb 128 2>/dev/null | tail -1 &&
timeout -k 10 300 python bench.py --workload resnet50_dgc --steps 30 --warmup 10 --exposed-steps 0 > gpurun_out/r3_dgc_bench.log 2>&1 && python3 tools/diag/benchline.py gpurun_out/r3_dgc_bench.log dgc
