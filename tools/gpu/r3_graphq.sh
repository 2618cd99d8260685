#!/bin/bash
# Round 3: how the HIP runtime executes the forked whole-step graph -- headline bench under the
# graph-execution knobs of the HIP runtime (host issue time per replay reported by bench.py).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
for cfg in ${CFGS:-"base A=1" "pkt1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "pkt0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "fq1 DEBUG_HIP_FORCE_GRAPH_QUEUES=1" "fq2 DEBUG_HIP_FORCE_GRAPH_QUEUES=2" "bs8 DEBUG_HIP_GRAPH_BATCH_SIZE=8" "inline GRACE_WGRAD_STREAM=0"}; do
  read -r tag envs <<< "$cfg"
  env $envs timeout -k 10 300 python bench.py --steps 30 --warmup 10 --grace-split off --exposed-steps 0 > gpurun_out/gq_$tag.log 2>&1 || { echo "$tag FAILED"; tail -3 gpurun_out/gq_$tag.log; continue; }
  python3 -c "
import json
for l in open('gpurun_out/gq_$tag.log'):
    if l.startswith('{\"metric'):
        d = json.loads(l); print('$tag', d['value'], d['ms_per_step'], 'host issue', d['host_issue_ms_per_step'])
"
done
