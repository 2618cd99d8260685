#!/bin/bash
# Round 4: side-stream weight gradients on/off -- throughput vs host issue time of the graph launch.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; mkdir -p gpurun_out
O=gpurun_out/r4_host_ab.txt; : > $O
ab() { local tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/host_$tag.log 2>&1 || { tail -20 gpurun_out/host_$tag.log; exit 1; }; echo "$tag $(grep -o '"value": [0-9.]*' gpurun_out/host_$tag.log) $(grep -o '"host_issue_ms_per_step": [0-9.]*' gpurun_out/host_$tag.log)" >> $O; tail -1 $O; }
ab side GRACE_X=1
ab inline GRACE_WGRAD_STREAM=0
ab side_b GRACE_X=1
ab inline_b GRACE_WGRAD_STREAM=0
