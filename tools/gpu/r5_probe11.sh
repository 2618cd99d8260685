#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=gpurun_out/probe11; mkdir -p $D
for v in "noev GRACE_BENCH_NO_STEP_EVENTS=1" "ev X=1"; do
  set -- $v; tag=$1; shift
  env GRACE_BENCH_LOSS_RECORD=1 "$@" timeout -k 10 300 python -u bench.py --workload bert_none --steps 30 --warmup 10 --grace-split off --exposed-steps 0 > $D/$tag.json 2> $D/$tag.err
  echo "$tag rc=$? $(grep -o '"final_loss": [^,]*\|"value": [0-9.]*' $D/$tag.json | tr '\n' ' ') $(grep '\[bench\] losses' $D/$tag.err | cut -c1-300)"
done
