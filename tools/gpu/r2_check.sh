#!/bin/bash
# Full GPU test suite + smoke + headline bench (round-end rehearsal of the driver's checks).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1; rc=$?
tail -4 gpurun_out/gputests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log &&
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench.log 2>&1 && grep '"metric"' gpurun_out/bench.log | cut -c1-300
