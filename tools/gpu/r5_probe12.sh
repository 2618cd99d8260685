#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=gpurun_out/probe12; mkdir -p $D
for v in "both" "attn_only" "hidden_only" "none" "both --sync" "both --sdpa-math"; do
  timeout -k 10 240 python -u tools/gpu/bert_graph_nosync.py --variant $v > $D/out.txt 2> $D/err.txt
  rc=$?; echo "rc=$rc $(cut -c1-330 $D/out.txt)"; [ $rc -eq 0 ] || { tail -3 $D/err.txt; exit 1; }
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_conv3x3.py tests/test_gpu_oob.py -x -q --timeout 250 --timeout-method thread > $D/conv.log 2>&1
echo "conv tests rc=$?"; tail -2 $D/conv.log
