#!/bin/bash
# In-situ A/B of the BN grid-shape knobs on the graphed headline step (interleaved runs).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=gpurun_out/bnknobs; mkdir -p $D
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py > $D/$n.log 2>&1 || { tail -5 $D/$n.log; return 1; }
  python3 -c "import json,sys; l=[x for x in open('$D/$n.log') if x.startswith('{')][-1]; print('$n', json.loads(l)['value'])"
}
if [ "$1" = "tb" ]; then  # second pass: target blocks only
  for rep in 1 2 3; do
    run base$rep GRACE_BN_VPT_MIN=8 && run tb1024_$rep GRACE_BN_TARGET_BLOCKS=1024 \
      && run tb2048_$rep GRACE_BN_TARGET_BLOCKS=2048 || exit 1
  done
  exit 0
fi
for rep in 1 2; do
  run base$rep GRACE_BN_VPT_MIN=8 && run vpt4_$rep GRACE_BN_VPT_MIN=4 && run tb1024_$rep GRACE_BN_TARGET_BLOCKS=1024 \
    && run vpt2_$rep GRACE_BN_VPT_MIN=2 || exit 1
done
