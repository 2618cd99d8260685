#!/bin/bash
# Round 4: whole GPU suite, then the headline and compressed-config sweep.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r4_full_t.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/r4_full_t.log
[ $rc -eq 0 ] || exit 1
bash tools/gpu/r4_sweep2.sh
