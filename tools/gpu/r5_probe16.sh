#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=gpurun_out/probe16; mkdir -p $D
for wl in bert_none bert_qsgd; do
  GRACE_BENCH_LOSS_RECORD=1 timeout -k 10 300 python -u bench.py --workload $wl --steps 30 --warmup 10 > $D/$wl.json 2> $D/$wl.err
  echo "$wl rc=$? $(grep -o '"final_loss": [^,]*\|"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"grace_ms_per_step": [0-9.]*' $D/$wl.json | tr '\n' ' ') $(grep '\[bench\] losses' $D/$wl.err | cut -c1-330)"
done
