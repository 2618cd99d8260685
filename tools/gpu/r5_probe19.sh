#!/bin/bash
# PowerSGD deferred residual: GPU numerics, exchange time on/off, kernel table; then the HIP
# graph-execution knob sweep on the headline.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=gpurun_out/probe19; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_compressors.py -x -q -k powersgd --timeout 250 --timeout-method thread > $D/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|^E  " $D/tests.log | head -6; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  GRACE_POWERSGD_DEFER_RESID=$v timeout -k 10 200 python -u benchmarks/grace_kernels.py --pipeline powersgd --iters 30 > $D/ex_$v.txt 2>&1 || exit 1
  echo "defer=$v $(grep -v amdgpu.ids $D/ex_$v.txt | tail -2 | tr '\n' ' ')"
done
bash tools/gpu/r2_prof_pipe.sh powersgd || exit 1
bash tools/gpu/r5_hipknobs.sh
