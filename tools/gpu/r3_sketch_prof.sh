#!/bin/bash
# Round 3: Sketch-64 ResNet-50 exchange kernel table (one 128 MB bucket, graph-replayed).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_sk" -o run -- \
  python3 "$R/benchmarks/grace_kernels.py" --pipeline sketch --iters 20 --bucket-mb 128 > "$R/gpurun_out/prof_sk.log" 2>&1 || exit 1
cd "$R" && tail -1 gpurun_out/prof_sk.log && python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_sk/**/*kernel_stats.csv", recursive=True) + glob.glob("gpurun_out/prof_sk/*kernel_stats.csv")
rows = list(csv.DictReader(open(f[0])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f'{float(r["TotalDurationNs"])/1e3:10.1f} us {int(r["Calls"]):6d} calls {float(r["AverageNs"])/1e3:8.2f} us/call  {r["Name"][:110]}')
PY
rm -f gpurun_out/prof_sk/*kernel_trace.csv
