#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/gpu/r3_graph_prof.sh r4ddp --surface ddp --warmup 12 > /dev/null 2>&1; head -45 gpurun_out/prof_r4ddp_steps.txt
