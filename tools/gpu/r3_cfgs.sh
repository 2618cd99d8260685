#!/bin/bash
# headline bench once per "tag ENV=V ..." argument (in order), one line each
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
for cfg in "$@"; do
  read -r tag envs <<< "$cfg"
  env $envs timeout -k 10 300 python bench.py --steps 30 --warmup 10 --grace-split off --exposed-steps 0 > gpurun_out/cf_$tag.log 2>&1 || { echo "$tag FAILED"; tail -3 gpurun_out/cf_$tag.log; exit 1; }
  python3 tools/diag/benchline.py gpurun_out/cf_$tag.log $tag
done
