R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bnact.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_bnact.log 2>&1; rc=$?; tail -4 gpurun_out/gpu_bnact.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python benchmarks/bnact_bench.py > gpurun_out/bnact_bench.txt 2>&1; cat gpurun_out/bnact_bench.txt &&
printf -- "--steps 30 --warmup 10\n--workload resnet50_none --steps 30 --warmup 10\n--workload resnet9_dawn --steps 30 --warmup 10\n" > gpurun_out/sw3.txt &&
bash tools/bench_sweep.sh gpurun_out/sw3.txt &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_bn -o run -- python3 $R/bench.py --steps 10 --warmup 5 > $R/gpurun_out/prof_bn.log 2>&1 && cd $R &&
python3 tools/prof_summary.py gpurun_out/prof_bn/run_kernel_trace.csv --steps 8 --marker Cijk_Alik_Bljk --per-step-markers 1 --top 45 > gpurun_out/prof_bn_summary.txt && rm -f gpurun_out/prof_bn/run_kernel_trace.csv && head -24 gpurun_out/prof_bn_summary.txt
