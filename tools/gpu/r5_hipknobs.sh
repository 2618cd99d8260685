#!/bin/bash
# HIP graph-execution knobs A/B on the fp32 ResNet-50 headline (forked whole-step graph):
# throughput and host issue time per replay for each runtime setting.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=gpurun_out/hipknobs; mkdir -p $D
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 170 python -u bench.py --steps 30 --warmup 10 > $D/$tag.json 2> $D/$tag.err
  local rc=$?
  echo "$tag rc=$rc $(grep -o '"value": [0-9.]*\|"host_issue_ms_per_step": [0-9.]*' $D/$tag.json | tr '\n' ' ')"
  return $rc
}
for v in "default" "DEBUG_HIP_FORCE_GRAPH_QUEUES=1" "DEBUG_HIP_FORCE_GRAPH_QUEUES=2" "DEBUG_HIP_FORCE_GRAPH_QUEUES=8" \
         "DEBUG_HIP_GRAPH_BATCH_SIZE=256" "DEBUG_CLR_MAX_BATCH_SIZE=256" "GRACE_WGRAD_STREAM=0"; do
  if [ "$v" = default ]; then run default GRACE_X=1 || exit 1; else run "$v" "$v" || exit 1; fi
done
