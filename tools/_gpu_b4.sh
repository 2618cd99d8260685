R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
timeout -k 10 200 python benchmarks/bnact_bench.py > gpurun_out/bnact_bench_graph.txt 2>&1; cat gpurun_out/bnact_bench_graph.txt &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_g -o run -- python3 $R/bench.py --steps 10 --warmup 5 > $R/gpurun_out/prof_g.log 2>&1 && cd $R &&
python3 tools/trace_by_grid.py gpurun_out/prof_g/run_kernel_trace.csv --match grace::bn_ --top 70 > gpurun_out/bn_by_grid.txt && rm -f gpurun_out/prof_g/run_kernel_trace.csv && cat gpurun_out/bn_by_grid.txt
