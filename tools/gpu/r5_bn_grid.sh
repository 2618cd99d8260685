#!/bin/bash
# Per-(kernel, grid) times of the GRACE kernels inside the graphed headline step's steady state
# (rocprofv3 kernel trace; the autotune calls before the window are excluded).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=gpurun_out/bngrid; mkdir -p $D
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/$D/prof" -o run -- \
  python3 "$R/bench.py" --steps 10 --warmup 5 > "$R/$D/prof.log" 2>&1 || exit 1
cd "$R"; f=$(find $D/prof -name "*kernel_trace.csv" | head -1)
python3 tools/prof_summary.py "$f" --steps 8 --marker topk2_split --per-step-markers 1 --top 5 \
  --grid-match "grace::" > $D/grid.txt && head -90 $D/grid.txt
rm -f "$f"
