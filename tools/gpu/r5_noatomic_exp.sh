R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=$R/gpurun_out/noat; mkdir -p $D
cd /tmp
for v in 0 1; do
  if [ $v = 1 ]; then export GRACE_PS_EXP_NOATOMIC=1; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $D/p$v -o run -- python3 $R/benchmarks/grace_kernels.py --pipeline powersgd --iters 10 --bucket-mb 128 > $D/p$v.log 2>&1 || exit 1
  f=$(find $D/p$v -name "*kernel_trace.csv" | head -1); echo "== noatomic=$v"; python3 $R/tools/trace_by_grid.py "$f" --match ps_mtp --top 4; rm -f "$f"
done
