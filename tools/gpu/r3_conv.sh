#!/bin/bash
# Round 3: autotuned 1x1 conv dispatch -- tests, the per-layer decision table, headline bench A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_conv.py > gpurun_out/r3_conv_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r3_conv_tests.log; [ $rc -eq 0 ] || exit $rc
GRACE_CONV_AUTO=0 timeout -k 10 300 python bench.py --steps 30 --warmup 10 --grace-split off > gpurun_out/r3_conv_off.log 2>&1 && grep -o '"value": [0-9.]*, "unit": "images/s", "n_gpus": 1, "steps": 30, "warmup": 10, "ms_per_step": [0-9.]*' gpurun_out/r3_conv_off.log &&
timeout -k 10 300 python -c "
import runpy, sys, json
sys.argv = ['bench.py', '--steps', '30', '--warmup', '10', '--grace-split', 'off']
try:
    runpy.run_path('bench.py', run_name='__main__')
finally:
    from grace_amd.ops import conv
    for r in conv.autotune_table():
        print('AUTOTUNE', r, flush=True)
" > gpurun_out/r3_conv_on.log 2>&1 && grep -o '"value": [0-9.]*, "unit": "images/s", "n_gpus": 1, "steps": 30, "warmup": 10, "ms_per_step": [0-9.]*' gpurun_out/r3_conv_on.log && grep AUTOTUNE gpurun_out/r3_conv_on.log | cut -c1-160
