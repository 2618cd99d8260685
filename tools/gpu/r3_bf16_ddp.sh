#!/bin/bash
# Round 3: bf16 (secondary) headline with / without the wgrad side stream; engine eager vs DDP
# comm-hook surface (eager and graph-captured).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_wgrad.py tests/test_gpu_bnact.py -k "not atomic" > gpurun_out/r3_bf_tests.log 2>&1; rc=$?
tail -1 gpurun_out/r3_bf_tests.log; [ $rc -eq 0 ] || exit $rc
b() { local tag=$1; shift; env $ENVS timeout -k 10 400 python bench.py --steps 30 --warmup 10 --grace-split off --exposed-steps 0 "$@" > gpurun_out/bd_$tag.log 2>&1 && python3 tools/diag/benchline.py gpurun_out/bd_$tag.log $tag || { echo "$tag FAILED"; tail -3 gpurun_out/bd_$tag.log; }; }
ENVS="A=1" b bf16_side --dtype bf16
ENVS="GRACE_WGRAD_STREAM=0" b bf16_inline --dtype bf16
ENVS="A=1" b engine_eager --graph off
ENVS="A=1" b ddp_eager --surface ddp
ENVS="A=1" b ddp_graph --surface ddp --graph full
