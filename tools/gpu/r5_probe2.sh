#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=gpurun_out/probe2; mkdir -p $D
timeout -k 10 120 python -u tools/gpu/bn_bwd_capture.py --force dgrad=mfma_t2 --variant pinned --modes plain_off,plain_on > $D/pinned.json 2> $D/pinned.err
rc=$?; echo "pinned rc=$rc"; python -c "
import json
for l in open('$D/pinned.json'):
    if not l.startswith('{'): continue
    d=json.loads(l); print(d['mode'], d['bn2_bias_rel_err'])
    for k in sorted(d):
        if k.startswith('bwd'): print('  ',k, {q: d[k][q] for q in ('db_vs_grad','db_vs_fp64','dy_sum_vs_fp64','db_rel')})
"; [ $rc -eq 0 ] || exit 1
for m in graph_fused; do
  for dp in 0.1 0.0; do
    timeout -k 10 300 python -u tools/gpu/bert_loss_trace.py --workload bert_none --modes $m --dropout $dp > $D/bert_${m}_$dp.json 2> $D/bert_${m}_$dp.err
    rc=$?; echo "bert $m dropout $dp rc=$rc"; cut -c1-600 $D/bert_${m}_$dp.json; tail -3 $D/bert_${m}_$dp.err | cut -c1-300
    [ $rc -eq 0 ] || exit 1
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse_decode.py tests/test_gpu_capacity_graph.py tests/test_gpu_xgmi.py -x -q --timeout 250 --timeout-method thread > $D/tests.log 2>&1
echo "tests rc=$?"; tail -3 $D/tests.log
