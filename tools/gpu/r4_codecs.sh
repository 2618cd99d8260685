#!/bin/bash
# Round 4: Sketch q > 1024, DGC fused compensate + depth-5 refinement: tests + exchange microbench.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sketch.py tests/test_gpu_compressors.py \
  tests/test_gpu_capacity_graph.py > gpurun_out/r4_codec_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r4_codec_tests.log; [ $rc -eq 0 ] || exit 1
O=gpurun_out/r4_codec_bench.txt; : > $O
for p in dgc topk sketch; do
  timeout -k 10 200 python benchmarks/grace_kernels.py --pipeline $p --iters 20 --bucket-mb 128 2>/dev/null | tail -1 >> $O || echo "grace_kernels $p failed" >> $O
done
cat $O
