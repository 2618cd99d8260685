R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t23.log 2>&1; echo T=$?; tail -3 gpurun_out/t23.log
bash tools/bench_sweep.sh tools/sweep23.txt || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof23_vgg -o run -- python3 $R/bench.py --workload vgg16_powersgd --steps 20 --warmup 5 --exposed-steps 0 > $R/gpurun_out/prof23_vgg.log 2>&1 || exit 1
cd $R && rm -f gpurun_out/prof23_vgg/run_kernel_trace.csv && python3 tools/prof_stats.py gpurun_out/prof23_vgg/run_kernel_stats.csv --top 3 --per 28 --grace
