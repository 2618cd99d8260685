#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=gpurun_out/probe3; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse_decode.py tests/test_gpu_capacity_graph.py -x -q --timeout 250 --timeout-method thread > $D/tests.log 2>&1
echo "tests rc=$?"; tail -2 $D/tests.log
for wl in bert_none bert_qsgd; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps 30 --warmup 10 > $D/bench_$wl.json 2> $D/bench_$wl.err
  rc=$?; echo "bench $wl rc=$rc"; grep -o '"value": [0-9.]*\|"final_loss": [^,]*\|"loss_finite": [a-z]*\|"ms_per_step": [0-9.]*' $D/bench_$wl.json | tr '\n' ' '; echo
  [ $rc -eq 0 ] || exit 1
done
timeout -k 10 400 python -u tools/gpu/bert_loss_trace.py --workload bert_none --modes eager_fused --steps 60 > $D/bert60.json 2> $D/bert60.err
echo "trace rc=$?"; cut -c1-900 $D/bert60.json
