#!/bin/bash
# full GPU test suite (one pytest process) + the convergence numbers + smoke
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -s > gpurun_out/gputests.log 2>&1; rc=$?
grep -E "passed|failed|error" gpurun_out/gputests.log | tail -3; grep -o "{'none'.*" gpurun_out/gputests.log | head -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -2 gpurun_out/smoke.log
