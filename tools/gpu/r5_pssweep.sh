#!/bin/bash
# PowerSGD kernel geometry sweep (VGG-16, 128 MB buckets as bench.py): ps_mq column strip and
# ps_mtp workgroup target.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=gpurun_out/pssweep; mkdir -p $D
for cfg in "2048 1024" "1024 1024" "4096 1024" "8192 1024" "2048 512" "2048 2048" "2048 4096"; do set -- $cfg
  GRACE_PS_MQ_COLS=$1 GRACE_PS_MTP_WG=$2 timeout -k 10 200 python -u benchmarks/grace_kernels.py --pipeline powersgd \
    --iters 30 --bucket-mb 128 > $D/s_$1_$2.txt 2>&1 || exit 1
  echo "cols=$1 mtp_wg=$2 $(grep -v amdgpu.ids $D/s_$1_$2.txt | tail -1)"
done
