#!/bin/bash
# Round 4 final check: build entry smoke, full GPU suite, the driver's default bench line.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4_smoke.log 2>&1 || { tail -20 gpurun_out/r4_smoke.log; exit 1; }
tail -1 gpurun_out/r4_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r4_final_t.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r4_final_t.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r4_final_bench.log 2>&1 || { tail -20 gpurun_out/r4_final_bench.log; exit 1; }
grep '"metric"' gpurun_out/r4_final_bench.log | cut -c1-300
