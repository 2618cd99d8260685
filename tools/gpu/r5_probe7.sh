#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=gpurun_out/probe7; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_oob.py -x -q --timeout 250 --timeout-method thread > $D/oob.log 2>&1
echo "oob rc=$?"; tail -2 $D/oob.log
GRACE_AUTOTUNE_REPORT=1 timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $D/bench.json 2> $D/bench.err
echo "bench rc=$?"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"host_issue_ms_per_step": [0-9.]*' $D/bench.json | tr '\n' ' '; echo
grep "^conv (" $D/bench.err | head -40
