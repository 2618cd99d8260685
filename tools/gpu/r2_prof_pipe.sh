#!/bin/bash
# rocprofv3 kernel stats of one grace_kernels pipeline.  Usage: r2_prof_pipe.sh PIPELINE
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
P=$1
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$P" -o run -- \
  python3 "$R/benchmarks/grace_kernels.py" --pipeline $P --iters 20 > "$R/gpurun_out/prof_$P.log" 2>&1 || exit 1
cd "$R"; f=$(find gpurun_out/prof_$P -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:25]: print('%10.1f us %6s calls %8.2f us/call  %s'%(float(r['TotalDurationNs'])/1e3, r['Calls'], float(r['AverageNs'])/1e3, r['Name'][:100]))
" | tee gpurun_out/prof_${P}_stats.txt
find gpurun_out/prof_$P -name "*kernel_trace.csv" -delete
