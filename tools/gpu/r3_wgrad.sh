#!/bin/bash
# Round 3: weight gradients on a side stream + autotuned dgrad form (ops/wgrad.py) -- tests, then
# the headline bench A/B (each configuration twice, alternating).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_wgrad.py > gpurun_out/r3_wgrad_tests.log 2>&1; rc=$?
tail -14 gpurun_out/r3_wgrad_tests.log; [ $rc -eq 0 ] || exit $rc
B='"value": [0-9.]*, "unit": "images/s", "n_gpus": 1, "steps": 30, "warmup": 10, "ms_per_step": [0-9.]*'
run() { local tag=$1; shift; echo "$tag:"; env "$@" timeout -k 10 300 python -c "
import runpy, sys
sys.argv = ['bench.py', '--steps', '30', '--warmup', '10', '--grace-split', 'off', '--exposed-steps', '0']
try:
    runpy.run_path('bench.py', run_name='__main__')
finally:
    from grace_amd.ops import wgrad
    for r in wgrad.dgrad_table():
        print('DGRAD', r, flush=True)
" > gpurun_out/r3_wg_$tag.log 2>&1 && grep -o "$B" gpurun_out/r3_wg_$tag.log; }
run inline GRACE_WGRAD_STREAM=0 GRACE_DGRAD_AUTO=0 &&
run side GRACE_DGRAD_AUTO=0 &&
run side_dgrad A=1 &&
run inline_b GRACE_WGRAD_STREAM=0 GRACE_DGRAD_AUTO=0 &&
run side_b GRACE_DGRAD_AUTO=0 &&
run side_dgrad_b A=1 && grep DGRAD gpurun_out/r3_wg_side_dgrad.log | cut -c1-200
