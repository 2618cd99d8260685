#!/bin/bash
# GPU-box sanity pass (run through gpurun): every GPU test, the driver's smoke(), the headline
# bench.  Each step bounded, chained so the first failure ends the call.
#   gpurun --timeout 1100 -- 'bash tools/gpu/check.sh'
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1; rc=$?
tail -3 gpurun_out/gputests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log &&
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log
