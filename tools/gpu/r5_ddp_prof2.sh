R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=$R/gpurun_out/ddpprof2; mkdir -p $D
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/ddp -o run -- python3 $R/bench.py --steps 10 --warmup 5 --surface ddp > $D/ddp.log 2>&1 || exit 1
cd $R && python3 tools/prof_summary.py $D/ddp/run_kernel_trace.csv --steps 8 --marker topk2_split --per-step-markers 1 --top 80 > $D/sum.txt && rm -f $D/ddp/run_kernel_trace.csv || exit 1
head -3 $D/sum.txt; grep -i "copy\|foreach\|multi_tensor\|gather_seg" $D/sum.txt
