#!/bin/bash
# Round 5 check: build-entry smoke, full GPU suite, the driver's default bench line, then the
# graphed headline kernel table.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=gpurun_out/r5final; mkdir -p $D
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $D/tests.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 400 python bench.py > $D/bench.log 2>&1 || { tail -20 $D/bench.log; exit 1; }
grep '"metric"' $D/bench.log | cut -c1-400
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/$D/prof" -o run -- \
  python3 "$R/bench.py" --steps 10 --warmup 5 > "$R/$D/prof.log" 2>&1 || exit 1
cd "$R" && python3 tools/prof_summary.py $D/prof/run_kernel_trace.csv --steps 8 --marker topk2_split \
  --per-step-markers 1 --top 45 > $D/prof_summary.txt && rm -f $D/prof/run_kernel_trace.csv && head -12 $D/prof_summary.txt
