R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
for O in fused torch; do
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_$O -o run -- python3 $R/bench.py --steps 10 --warmup 5 --optimizer $O > $R/gpurun_out/prof_$O.log 2>&1 || exit 1
cd $R && python3 tools/prof_summary.py gpurun_out/prof_$O/run_kernel_trace.csv --steps 8 --marker Cijk_Alik_Bljk --per-step-markers 1 --top 12 > gpurun_out/prof_${O}_summary.txt && python3 tools/trace_by_grid.py gpurun_out/prof_$O/run_kernel_trace.csv --match sgd --top 10 >> gpurun_out/prof_${O}_summary.txt; python3 tools/trace_by_grid.py gpurun_out/prof_$O/run_kernel_trace.csv --match multi_tensor --top 10 >> gpurun_out/prof_${O}_summary.txt; python3 tools/trace_by_grid.py gpurun_out/prof_$O/run_kernel_trace.csv --match cast_segments --top 10 >> gpurun_out/prof_${O}_summary.txt; rm -f gpurun_out/prof_$O/run_kernel_trace.csv; cat gpurun_out/prof_${O}_summary.txt
done
