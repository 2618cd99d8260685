#!/bin/bash
# Round 3: Sketch q >= 128 native select tests + chunk-size sweep of the Sketch(64) exchange.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_sketch.py > gpurun_out/r3_sketch_tests.log 2>&1; rc=$?
tail -15 gpurun_out/r3_sketch_tests.log; [ $rc -eq 0 ] || exit $rc
for qc in 65536 32768 16384; do for cc in 32768 8192 4096; do
  echo "qsel $qc codec $cc: $(GRACE_QSEL_CHUNK=$qc GRACE_CODEC_CHUNK=$cc timeout -k 10 120 python benchmarks/grace_kernels.py --pipeline sketch --model resnet50 --iters 20 --bucket-mb 128 2>/dev/null | tail -1)" || exit 1
done; done
