#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
for cfg in "base A=1" "cpwait GPU_STREAMOPS_CP_WAIT=1" "fq4 DEBUG_HIP_FORCE_GRAPH_QUEUES=4" "prio_hi GRACE_WGRAD_PRIORITY=-1" "async DEBUG_HIP_FORCE_ASYNC_QUEUE=1"; do
  read -r tag envs <<< "$cfg"
  env $envs timeout -k 10 300 python bench.py --steps 30 --warmup 10 --grace-split off --exposed-steps 0 > gpurun_out/gq_$tag.log 2>&1 || { echo "$tag FAILED"; tail -3 gpurun_out/gq_$tag.log; continue; }
  python3 -c "
import json
for l in open('gpurun_out/gq_$tag.log'):
    if l.startswith('{\"metric'):
        d = json.loads(l); print('$tag', d['value'], d['ms_per_step'], 'host issue', d['host_issue_ms_per_step'])
"
done
