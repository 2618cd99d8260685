#!/bin/bash
# Bit-packed small-s QSGD codes: GPU compressor/property tests, W=2 multi-rank GPU tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_compressors.py tests/test_properties.py tests/test_gpu_multirank.py -m gpu -x -q --timeout 240 --timeout-method thread \
  > gpurun_out/qsgd_pack_tests.log 2>&1; rc=$?; tail -2 gpurun_out/qsgd_pack_tests.log; exit $rc
