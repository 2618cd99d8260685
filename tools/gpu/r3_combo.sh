#!/bin/bash
# Round 3 combo: sketch / conv / BN GPU tests, autotuned-conv + BN-dz bench A/B, sketch chunk sweep.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_sketch.py tests/test_gpu_conv.py tests/test_gpu_bnact.py > gpurun_out/r3_combo_tests.log 2>&1; rc=$?
tail -4 gpurun_out/r3_combo_tests.log; [ $rc -eq 0 ] || exit $rc
B='"value": [0-9.]*, "unit": "images/s", "n_gpus": 1, "steps": 30, "warmup": 10, "ms_per_step": [0-9.]*'
echo "conv auto OFF, bn dz OFF:" && GRACE_CONV_AUTO=0 GRACE_BN_DZ=0 timeout -k 10 300 python bench.py --steps 30 --warmup 10 --grace-split off > gpurun_out/r3_ab0.log 2>&1 && grep -o "$B" gpurun_out/r3_ab0.log &&
echo "conv auto OFF, bn dz ON:" && GRACE_CONV_AUTO=0 timeout -k 10 300 python bench.py --steps 30 --warmup 10 --grace-split off > gpurun_out/r3_ab1.log 2>&1 && grep -o "$B" gpurun_out/r3_ab1.log &&
echo "conv auto ON, bn dz ON:" && timeout -k 10 300 python -c "
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
" > gpurun_out/r3_ab2.log 2>&1 && grep -o "$B" gpurun_out/r3_ab2.log && grep -E "AUTOTUNE|BNTUNE" gpurun_out/r3_ab2.log | cut -c1-220 || exit 1
timeout -k 10 200 python benchmarks/gemm_bench.py --iters 20 2>/dev/null | tee gpurun_out/r3_gemm_bench.txt || exit 1
for cfg in "65536 32768" "32768 8192" "16384 8192" "16384 4096"; do set -- $cfg
  echo "sketch qsel $1 codec $2: $(GRACE_QSEL_CHUNK=$1 GRACE_CODEC_CHUNK=$2 timeout -k 10 120 python benchmarks/grace_kernels.py --pipeline sketch --model resnet50 --iters 20 --bucket-mb 128 2>/dev/null | tail -1)" || exit 1
done
