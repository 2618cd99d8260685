#!/bin/bash
# decode / wgrad tests after the one-launch decode removal, DGC + PowerSGD exchange kernel tables,
# then the HIP graph-execution knob sweep on the headline.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=gpurun_out/probe18; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_sparse_decode.py tests/test_gpu_wgrad.py -x -q \
  -W "error:The AccumulateGrad node's stream:UserWarning" --timeout 250 --timeout-method thread > $D/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|^E  " $D/tests.log | head -6; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/r2_prof_pipe.sh dgc || exit 1
bash tools/gpu/r2_prof_pipe.sh powersgd || exit 1
bash tools/gpu/r5_hipknobs.sh
