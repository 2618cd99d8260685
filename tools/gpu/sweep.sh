#!/bin/bash
# bench.py runs on the GPU box, one per argument (see tools/bench_sweep.sh), output appended to
# gpurun_out/sweep.txt.   gpurun --timeout 900 -- 'bash tools/gpu/sweep.sh "--steps 30" "--surface ddp"'
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/bench_sweep.sh -- "$@" | tee -a gpurun_out/sweep.txt
exit ${PIPESTATUS[0]}
