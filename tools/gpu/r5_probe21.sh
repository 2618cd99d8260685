#!/bin/bash
# DGC compaction A/B (masks / plain read) and the PowerSGD exchange kernels per grid (128 MB buckets, as bench.py).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=gpurun_out/probe21; mkdir -p $D
timeout -k 10 200 python -u tools/gpu/dgc_compact_ab.py 2>&1 | grep -v amdgpu.ids || exit 1
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$R/$D/ps" -o run -- \
  python3 "$R/benchmarks/grace_kernels.py" --pipeline powersgd --iters 10 --bucket-mb 128 > "$R/$D/ps.log" 2>&1 || exit 1
cd "$R"; f=$(find $D/ps -name "*kernel_trace.csv" | head -1)
python3 tools/trace_by_grid.py "$f" --match grace:: --top 40 | tee $D/ps_grid.txt
rm -f "$f"
