#!/bin/bash
# Sketch encode: which part of the per-element work costs the time (GRACE_SKETCH_DBG modes)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONUNBUFFERED=1 GRACE_SKETCH_PROBE_QUICK=1; mkdir -p gpurun_out
: > gpurun_out/sk3_probe.log
for d in 0; do
  GRACE_SKETCH_DBG=$d timeout -k 10 120 python tools/diag/sketch_encode_probe.py 2>&1 | grep "us$" >> gpurun_out/sk3_probe.log || exit 1
done
cat gpurun_out/sk3_probe.log
