#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; mkdir -p gpurun_out
O=gpurun_out/r4_c3onoff.txt; : > $O
ab() { local tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 30 --warmup 10 $W > gpurun_out/c3oo_$tag.log 2>&1 || { tail -20 gpurun_out/c3oo_$tag.log; exit 1; }; echo "$tag $(grep -o '"value": [0-9.]*' gpurun_out/c3oo_$tag.log)" >> $O; tail -1 $O; }
W=""; ab topk_on GRACE_X=1; ab topk_off GRACE_CONV3X3=0; ab topk_on_b GRACE_X=1; ab topk_off_b GRACE_CONV3X3=0
W="--workload resnet50_none"; ab none_on GRACE_X=1; ab none_off GRACE_CONV3X3=0
