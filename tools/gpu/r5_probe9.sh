#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=gpurun_out/probe9; mkdir -p $D
run() {  # tag, env..., -- bench args
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --workload bert_none --steps 30 --warmup 10 --grace-split off --exposed-steps 0 > $D/$tag.json 2> $D/$tag.err
  local rc=$?; echo "$tag rc=$rc $(grep -o '"final_loss": [^,]*\|"value": [0-9.]*' $D/$tag.json | tr '\n' ' ')"; return $rc
}
run base X=1 && run sync_each GRACE_GRAPH_SYNC_EACH=1 && true
for v in "torch_sgd --optimizer torch" "graph_off --graph off"; do
  set -- $v; tag=$1; shift
  timeout -k 10 300 python -u bench.py --workload bert_none --steps 30 --warmup 10 --grace-split off --exposed-steps 0 "$@" > $D/$tag.json 2> $D/$tag.err
  echo "$tag rc=$? $(grep -o '"final_loss": [^,]*\|"value": [0-9.]*' $D/$tag.json | tr '\n' ' ')"
done
