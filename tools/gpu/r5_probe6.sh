#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=gpurun_out/probe6; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_xgmi.py -x -q --timeout 250 --timeout-method thread -k "matches_eager" > $D/rehearsal.log 2>&1
echo "rehearsal rc=$?"; grep -E "passed|failed|^E  " $D/rehearsal.log | head -8
for b in "" "--benchmark"; do
  timeout -k 10 300 python -u tools/gpu/bert_loss_trace.py --workload bert_none --modes graph_fused --steps 60 --cap-warm 5 $b > $D/bert_graph$b.json 2> $D/bert_graph$b.err
  echo "bert graph $b rc=$?"; cut -c1-1200 $D/bert_graph$b.json
done
