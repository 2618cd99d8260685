#!/bin/bash
# Round 3: weight gradients on a side stream (ops/wgrad.py) -- tests, then the headline bench A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_wgrad.py > gpurun_out/r3_wgrad_tests.log 2>&1; rc=$?
tail -8 gpurun_out/r3_wgrad_tests.log; [ $rc -eq 0 ] || exit $rc
B='"value": [0-9.]*, "unit": "images/s", "n_gpus": 1, "steps": 30, "warmup": 10, "ms_per_step": [0-9.]*'
echo "wgrad in line:" && GRACE_WGRAD_STREAM=0 timeout -k 10 300 python bench.py --steps 30 --warmup 10 --grace-split off --exposed-steps 0 > gpurun_out/r3_wg0.log 2>&1 && grep -o "$B" gpurun_out/r3_wg0.log &&
echo "wgrad side stream:" && timeout -k 10 300 python bench.py --steps 30 --warmup 10 --grace-split off --exposed-steps 0 > gpurun_out/r3_wg1.log 2>&1 && grep -o "$B" gpurun_out/r3_wg1.log &&
echo "wgrad in line (again):" && GRACE_WGRAD_STREAM=0 timeout -k 10 300 python bench.py --steps 30 --warmup 10 --grace-split off --exposed-steps 0 > gpurun_out/r3_wg2.log 2>&1 && grep -o "$B" gpurun_out/r3_wg2.log &&
echo "wgrad side stream (again):" && timeout -k 10 300 python bench.py --steps 30 --warmup 10 --grace-split off --exposed-steps 0 > gpurun_out/r3_wg3.log 2>&1 && grep -o "$B" gpurun_out/r3_wg3.log
