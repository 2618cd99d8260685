#!/bin/bash
# Round 3: kernel trace of the GRAPHED fp32 headline step (wgrad side stream on): busy time,
# idle gaps, per-kernel table; then bench A/B of the GRACE exchange overlap / bucket size.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=${1:-r3g}
shift  # further arguments go to bench.py (e.g. --dtype bf16)
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof_$TAG" -o run -- \
  python3 "$R/bench.py" --steps 10 --warmup 6 --exposed-steps 0 --grace-split off "$@" > "$R/gpurun_out/prof_$TAG.log" 2>&1 || exit 1
cd "$R" && python3 tools/prof_summary.py gpurun_out/prof_$TAG/run_kernel_trace.csv --steps 8 --marker nll_loss_forward \
  --per-step-markers 1 --top 60 --gaps 25 > gpurun_out/prof_${TAG}_steps.txt &&
python3 tools/trace_seq.py gpurun_out/prof_$TAG/run_kernel_trace.csv > gpurun_out/prof_${TAG}_allseq.txt &&
python3 tools/trace_streams.py gpurun_out/prof_$TAG/run_kernel_trace.csv --steps 8 --tail 40 > gpurun_out/prof_${TAG}_streams.txt || exit 1
head -12 gpurun_out/prof_${TAG}_streams.txt
python3 -c "
import csv, gzip, sys
rows = csv.DictReader(open('gpurun_out/prof_$TAG/run_kernel_trace.csv'))
with gzip.open('gpurun_out/prof_${TAG}_trace.csv.gz', 'wt') as f:
    w = csv.writer(f)
    w.writerow(['Start_Timestamp', 'End_Timestamp', 'Queue_Id', 'Stream_Id', 'Kernel_Name'])
    for r in rows:
        w.writerow([r['Start_Timestamp'], r['End_Timestamp'], r.get('Queue_Id', ''), r.get('Stream_Id', ''), r['Kernel_Name'][:120]])
" && rm -f gpurun_out/prof_$TAG/run_kernel_trace.csv; head -40 gpurun_out/prof_${TAG}_steps.txt
