#!/bin/bash
# Generic headline A/B: each argument is "tag ENV=V ..." ; runs them in order, twice (alternating).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
B='"value": [0-9.]*, "unit": "images/s", "n_gpus": 1, "steps": 30, "warmup": 10, "ms_per_step": [0-9.]*'
for pass in a b; do
  for cfg in "$@"; do
    read -r tag envs <<< "$cfg"
    echo "$tag ($pass):"
    env $envs timeout -k 10 300 python bench.py --steps 30 --warmup 10 --grace-split off --exposed-steps 0 > gpurun_out/ab_${tag}_$pass.log 2>&1 || { tail -5 gpurun_out/ab_${tag}_$pass.log; exit 1; }
    grep -o "$B" gpurun_out/ab_${tag}_$pass.log
  done
done
