#!/bin/bash
# ps_mtp rows-per-batch A/B, then the VGG-16 PowerSGD bench line (in-step grace_ms).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=$R/gpurun_out/pspb; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_compressors.py -x -q -k "powersgd" --timeout 250 --timeout-method thread > $D/tests.log 2>&1 \
  || { tail -20 $D/tests.log; exit 1; }
for pb in 8 8; do
  echo "pb=$pb $(GRACE_PS_MTP_PB=$pb timeout -k 10 200 python -u benchmarks/grace_kernels.py --pipeline powersgd --iters 30 --bucket-mb 128 2>&1 | tail -1)" || exit 1
done
timeout -k 10 400 python -u bench.py --workload vgg16_powersgd --steps 20 --warmup 10 > $D/vgg.json 2> $D/vgg.err || exit 1
grep -o '"value": [0-9.]*\|"grace_ms_per_step": [0-9.]*\|"final_loss": [0-9.]*' $D/vgg.json | tr '\n' ' '
