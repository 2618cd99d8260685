#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; mkdir -p gpurun_out/bnrace
for v in none keep sync_before sync_after dummy_before; do
  timeout -k 10 100 python -u tools/gpu/bn_bwd_capture.py --force dgrad=mfma_t2 --variant $v --modes ddp_off,plain_on > gpurun_out/bnrace/$v.json 2> gpurun_out/bnrace/$v.err || exit 1
  echo "$v: $(grep -o '"mode": "[a-z_]*"\|"bn2_bias_rel_err": [0-9.e+-]*\|"kept0": {[^}]*}' gpurun_out/bnrace/$v.json | tr '\n' ' ')"
done
GRACE_BN_DETERMINISTIC=1 timeout -k 10 100 python -u tools/gpu/bn_bwd_capture.py --force dgrad=mfma_t2 --variant keep --modes ddp_off,plain_on > gpurun_out/bnrace/det_keep.json 2> gpurun_out/bnrace/det.err || exit 1
echo "det keep: $(grep -o '"mode": "[a-z_]*"\|"bn2_bias_rel_err": [0-9.e+-]*\|"kept0": {[^}]*}' gpurun_out/bnrace/det_keep.json | tr '\n' ' ')"
AMD_SERIALIZE_KERNEL=3 timeout -k 10 100 python -u tools/gpu/bn_bwd_capture.py --force dgrad=mfma_t2 --variant none --modes ddp_off,plain_on > gpurun_out/bnrace/serial.json 2> gpurun_out/bnrace/serial.err || exit 1
echo "serialize: $(grep -o '"mode": "[a-z_]*"\|"bn2_bias_rel_err": [0-9.e+-]*' gpurun_out/bnrace/serial.json | tr '\n' ' ')"
