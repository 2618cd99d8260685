# job 2: GRACE microbench, DAWN workload, headline kernel trace, PMC passes on the GRACE kernels
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
timeout -k 10 300 python -u benchmarks/grace_kernels.py --pipeline all > gpurun_out/grace_kernels.txt 2>&1 && cat gpurun_out/grace_kernels.txt &&
printf -- "--workload resnet9_dawn --steps 30 --warmup 10\n--workload resnet9_dawn --steps 30 --warmup 10 --bf16-weights off\n" > gpurun_out/sw2.txt &&
bash tools/bench_sweep.sh gpurun_out/sw2.txt &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_head -o run -- python3 $R/bench.py --steps 10 --warmup 5 > $R/gpurun_out/prof_head.log 2>&1 && cd $R &&
python3 tools/prof_summary.py gpurun_out/prof_head/run_kernel_trace.csv --steps 8 --marker Cijk_Alik_Bljk --per-step-markers 1 --top 45 > gpurun_out/prof_head_summary.txt && rm -f gpurun_out/prof_head/run_kernel_trace.csv && head -60 gpurun_out/prof_head_summary.txt &&
for P in topk powersgd; do
  cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES --output-format csv -d $R/gpurun_out/pmc_${P}_a -o run -- python3 $R/benchmarks/grace_kernels.py --pipeline $P --iters 2 --no-graph > $R/gpurun_out/pmc_${P}_a.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_${P}_b -o run -- python3 $R/benchmarks/grace_kernels.py --pipeline $P --iters 2 --no-graph > $R/gpurun_out/pmc_${P}_b.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_${P}_c -o run -- python3 $R/benchmarks/grace_kernels.py --pipeline $P --iters 2 --no-graph > $R/gpurun_out/pmc_${P}_c.log 2>&1 || exit 1
  cd $R && python3 tools/pmc_summary.py $(find gpurun_out/pmc_${P}_? -name '*counter_collection.csv') --grace > gpurun_out/pmc_${P}_summary.txt || exit 1
  cat gpurun_out/pmc_${P}_summary.txt
done
