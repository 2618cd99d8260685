#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=gpurun_out/probe10; mkdir -p $D
for v in "rec X=1" "rec_nodrop GRACE_BERT_DROPOUT=0.0" "rec_copies2 GRACE_GRAPH_COPIES=2"; do
  set -- $v; tag=$1; shift
  env GRACE_BENCH_LOSS_RECORD=1 "$@" timeout -k 10 300 python -u bench.py --workload bert_none --steps 30 --warmup 10 --grace-split off --exposed-steps 0 > $D/$tag.json 2> $D/$tag.err
  echo "$tag rc=$? $(grep -o '"final_loss": [^,]*' $D/$tag.json) $(grep '\[bench\] losses' $D/$tag.err | cut -c1-400)"
done
