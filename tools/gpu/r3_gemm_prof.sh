#!/bin/bash
# Round 3: fp32 GEMM throughput (MFMA GEMM vs hipBLASLt) + PMC counters of the MFMA GEMM on one
# memory-heavy and one compute-heavy 1x1-conv shape.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out/gemm_pmc
timeout -k 10 300 python benchmarks/gemm_bench.py --iters 20 > gpurun_out/r3_gemm_bench.txt 2>&1; rc=$?
cat gpurun_out/r3_gemm_bench.txt | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
cat > /tmp/gemm_one.py <<'PY'
import sys, torch
sys.path.insert(0, ".")
from grace_amd.ops.conv import gemm
m, cin, cout = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
x = torch.randn(m, cin, device="cuda"); wt = torch.randn(cout, cin, device="cuda"); y = torch.empty(m, cout, device="cuda")
for _ in range(5):
    gemm(x, True, cin, wt, True, cin, y, cout, m, cout, cin, 0)
torch.cuda.synchronize()
PY
for shp in "100352 64 256" "6272 1024 256"; do set -- $shp
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT -d gpurun_out/gemm_pmc/p1_$1 -o pmc -- python3 /tmp/gemm_one.py $1 $2 $3 > /dev/null 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_IDX_ACTIVE -d gpurun_out/gemm_pmc/p2_$1 -o pmc -- python3 /tmp/gemm_one.py $1 $2 $3 > /dev/null 2>&1 || exit 1
done
find gpurun_out/gemm_pmc -name "*counter_collection.csv" | head
