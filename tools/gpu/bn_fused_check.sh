#!/bin/bash
# Single-launch BN kernels + inline RCCL comm: BN GPU tests, per-shape graph timing, headline
# bench with the single-launch path on/off, and the RCCL-in-graph path (--force-dist) with the
# torch and native-inline comms.
#   gpurun --timeout 900 -- 'bash tools/gpu/bn_fused_check.sh'
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bnact.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/bn_tests.log 2>&1; rc=$?; tail -3 gpurun_out/bn_tests.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --steps 30 --warmup 10"
val() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["hip_graph"], d["config"].get("comm"))'; }
timeout -k 10 240 $B > gpurun_out/b_fused.log 2>&1 && echo "fused $(val gpurun_out/b_fused.log)" &&
GRACE_BN_FUSED=0 timeout -k 10 240 $B > gpurun_out/b_twokernel.log 2>&1 && echo "two-kernel $(val gpurun_out/b_twokernel.log)" &&
timeout -k 10 240 $B --force-dist > gpurun_out/b_fd_auto.log 2>&1 && echo "force-dist auto $(val gpurun_out/b_fd_auto.log)" &&
timeout -k 10 240 $B --force-dist --comm torch > gpurun_out/b_fd_torch.log 2>&1 && echo "force-dist torch $(val gpurun_out/b_fd_torch.log)" &&
timeout -k 10 240 python benchmarks/bnact_bench.py > gpurun_out/bn_shapes.txt 2>&1 && tail -20 gpurun_out/bn_shapes.txt &&
python -c "import grace_amd.ops._native as n; print('spin timeouts', n.lib().bn_spin_timeouts())"
