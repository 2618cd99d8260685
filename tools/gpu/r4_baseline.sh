#!/bin/bash
# Round 4 start: GPU test suite, headline bench, graphed kernel trace of the headline step.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_gputests.log 2>&1
echo "pytest rc=$?"; tail -3 gpurun_out/r4_gputests.log
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/r4_bench0.log 2>&1 || { echo bench failed; tail -5 gpurun_out/r4_bench0.log; exit 1; }
tail -1 gpurun_out/r4_bench0.log
bash tools/gpu/r3_graph_prof.sh r4base > /dev/null 2>&1; head -60 gpurun_out/prof_r4base_steps.txt
