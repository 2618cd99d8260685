R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof29 -o run -- python3 $R/bench.py --workload resnet50_topk --steps 10 --warmup 5 > $R/gpurun_out/prof29.log 2>&1 || exit 1
cd $R && python3 tools/prof_summary.py gpurun_out/prof29/run_kernel_trace.csv --steps 8 --marker Cijk_Alik_Bljk --per-step-markers 1 --top 45 > gpurun_out/prof29_summary.txt; rm -f gpurun_out/prof29/run_kernel_trace.csv; cat gpurun_out/prof29_summary.txt
