#!/bin/bash
# PMC counters of the f32 MFMA implicit-GEMM 3x3 data gradient vs MIOpen's solver on the ResNet-50
# 14x14x256 and 7x7x512 layers (batch 32): MFMA busy, wait, LDS and instruction mix.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=$R/gpurun_out/c3pmc; mkdir -p $D
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT"
P2="GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU"
cd /tmp
for cfg in "32 256 14 14 1 4 1" "32 256 14 14 1 -1 1" "32 512 7 7 1 2 4" "32 512 7 7 1 4 1" "32 512 7 7 1 -1 1"; do
  tag=$(echo $cfg | tr ' ' '_')
  timeout -k 10 60 python3 $R/tools/gpu/c3_pmc_one.py $cfg 20 2>&1 | grep -v amdgpu.ids || exit 1
  timeout -s KILL 60 rocprofv3 --pmc $P1 --output-format csv -d $D/p1_$tag -o run -- python3 $R/tools/gpu/c3_pmc_one.py $cfg 5 > /dev/null 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc $P2 --output-format csv -d $D/p2_$tag -o run -- python3 $R/tools/gpu/c3_pmc_one.py $cfg 5 > /dev/null 2>&1 || exit 1
  python3 $R/tools/pmc_summary.py $(find $D/p1_$tag $D/p2_$tag -name '*counter_collection.csv') --top 6 > $D/sum_$tag.txt || exit 1
  echo "== $cfg"; cat $D/sum_$tag.txt | cut -c1-260
done
