#!/bin/bash
# PowerSGD P = M Q with the Q rows staged through LDS: numerics, exchange time, per-grid kernel times.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=$R/gpurun_out/psstage; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_compressors.py tests/test_powersgd_step.py -x -q -k "powersgd or deferred or materialises" \
  --timeout 250 --timeout-method thread > $D/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|^E  " $D/tests.log | head -6; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 200 python -u benchmarks/grace_kernels.py --pipeline powersgd --iters 30 --bucket-mb 128 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1; done
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $D/ps -o run -- \
  python3 $R/benchmarks/grace_kernels.py --pipeline powersgd --iters 10 --bucket-mb 128 > $D/ps.log 2>&1 || exit 1
cd $R; f=$(find $D/ps -name "*kernel_trace.csv" | head -1)
python3 tools/trace_by_grid.py "$f" --match grace:: --top 14 | tee $D/ps_grid.txt; rm -f "$f"
