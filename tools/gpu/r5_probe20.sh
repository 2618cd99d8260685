#!/bin/bash
# DGC scanned compaction: numerics (compressors, capacity-graph, DGC-using tests), exchange time, kernel table.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=gpurun_out/probe20; mkdir -p $D
timeout -k 10 500 python -u -m pytest tests/test_gpu_compressors.py tests/test_gpu_capacity_graph.py tests/test_gpu_graph_rng.py -x -q \
  --timeout 250 --timeout-method thread > $D/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|^E  " $D/tests.log | head -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u benchmarks/grace_kernels.py --pipeline dgc --iters 30 --bucket-mb 128 > $D/ex.txt 2>&1 || exit 1
grep -v amdgpu.ids $D/ex.txt | tail -2
bash tools/gpu/r2_prof_pipe.sh dgc
