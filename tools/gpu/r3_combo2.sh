#!/bin/bash
# Round 3: DGC tree refinement (tests + microbench + bench) and round-robin graph copies A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/gpu/r3_dgc.sh || exit 1
bash tools/gpu/r3_cfgs.sh "copies1 A=1" "copies2 GRACE_GRAPH_COPIES=2" "copies3 GRACE_GRAPH_COPIES=3" "copies1_b A=1"
