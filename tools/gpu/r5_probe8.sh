#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=gpurun_out/probe8; mkdir -p $D
GRACE_BENCH_LOSS_TRACE=1 timeout -k 10 300 python -u bench.py --workload bert_none --steps 30 --warmup 10 > $D/bench_bert.json 2> $D/bench_bert.err
echo "bench bert rc=$?"; grep "\[bench\]" $D/bench_bert.err | tr '\n' ' ' | cut -c1-2500; echo
timeout -k 10 400 python -u -m pytest tests/test_gpu_xgmi.py -q --timeout 250 --timeout-method thread -k "matches_eager" > $D/rehearsal.log 2>&1
echo "rehearsal rc=$?"; grep -E "passed|failed|^E  " $D/rehearsal.log | head -8
