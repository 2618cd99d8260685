#!/bin/bash
# Round 3: conv bias backward through atomic totals -- convact tests + VGG-16 PowerSGD A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_convact.py tests/test_gpu_bnact.py > gpurun_out/vgg_tests.log 2>&1; rc=$?
tail -1 gpurun_out/vgg_tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in "atomic A=1" "tree GRACE_BN_ATOMIC_CHUNKS=0"; do
  read -r tag envs <<< "$cfg"
  env $envs timeout -k 10 400 python bench.py --workload vgg16_powersgd --steps 20 --warmup 10 --grace-split off --exposed-steps 0 > gpurun_out/vgg_$tag.log 2>&1 && python3 tools/diag/benchline.py gpurun_out/vgg_$tag.log vgg_$tag || { echo "$tag failed"; tail -3 gpurun_out/vgg_$tag.log; exit 1; }
done
