#!/bin/bash
# Two-level BN statistics fold: conv/BN GPU tests, per-piece conv->BN microbench, headline bench with tune tables.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=${1:-fold}
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_bnact.py > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -4 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/conv_bn_bench.py --iters 20 > gpurun_out/${TAG}_convbn.txt 2>&1; rc=$?
cat gpurun_out/${TAG}_convbn.txt; [ $rc -eq 0 ] || exit $rc
B='"value": [0-9.]*, "unit": "images/s", "n_gpus": 1, "steps": 30, "warmup": 10, "ms_per_step": [0-9.]*'
timeout -k 10 300 python -c "
import runpy, sys
sys.argv = ['bench.py', '--steps', '30', '--warmup', '10', '--grace-split', 'off']
try:
    runpy.run_path('bench.py', run_name='__main__')
finally:
    from grace_amd.ops import conv
    for r in conv.autotune_table():
        print('AUTOTUNE', r, flush=True)
    for r in conv.bn_autotune_table():
        print('BNTUNE', r, flush=True)
" > gpurun_out/${TAG}_bench.log 2>&1 && grep -o "$B" gpurun_out/${TAG}_bench.log && grep -E "BNTUNE" gpurun_out/${TAG}_bench.log | cut -c1-260
