#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=gpurun_out/probe14; mkdir -p $D
for v in "both --sync-at 9" "both --sync-at 3" "none --sync-at 9" "attn_only --sync-at 9" "hidden_only --sync-at 9"; do
  timeout -k 10 240 python -u tools/gpu/bert_graph_nosync.py --variant $v > $D/out.txt 2> $D/err.txt
  rc=$?; echo "rc=$rc $(cut -c1-260 $D/out.txt)"; [ $rc -eq 0 ] || { tail -3 $D/err.txt; exit 1; }
done
