#!/bin/bash
# Round 3: GPU tests of the comm hardening (RCCL self-check + concurrent issue, xGMI timeout /
# count-aware / direct slot, FusedSGD fault guard) + PowerSGD kernels + short benches.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_a_comm.py tests/test_gpu_xgmi.py "tests/test_gpu_compressors.py" -k "comm or xgmi or rccl or powersgd or ddp" > gpurun_out/r3_comm_tests.log 2>&1; rc=$?
tail -25 gpurun_out/r3_comm_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 10 > gpurun_out/r3_bench1.log 2>&1 && grep '"metric"' gpurun_out/r3_bench1.log | cut -c1-300 && grep -o '"grace_ms_per_step.*' gpurun_out/r3_bench1.log | cut -c1-200 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 10 --surface ddp > gpurun_out/r3_bench_ddp.log 2>&1 && grep '"metric"' gpurun_out/r3_bench_ddp.log | cut -c1-200 && grep -o '"hip_graph.*' gpurun_out/r3_bench_ddp.log | cut -c1-300
