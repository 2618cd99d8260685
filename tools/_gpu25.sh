R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/t25.log 2>&1; echo T=$?; grep -E "passed|failed|Error" gpurun_out/t25.log | tail -8
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof25_bert -o run -- python3 $R/bench.py --workload bert_qsgd --steps 20 --warmup 5 --exposed-steps 0 > $R/gpurun_out/prof25_bert.log 2>&1 || exit 1
cd $R && rm -f gpurun_out/prof25_bert/run_kernel_trace.csv && python3 tools/prof_stats.py gpurun_out/prof25_bert/run_kernel_stats.csv --top 8 --per 28 --grace | tee profiles/r1_bert_qsgd_after_fold_fix_stats.txt
