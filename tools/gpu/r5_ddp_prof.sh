#!/bin/bash
# Graphed kernel tables: DDP comm-hook surface vs the engine without the side-stream fork (same in-line wgrads).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=$R/gpurun_out/ddpprof; mkdir -p $D
for v in ddp nofork; do
  if [ $v = ddp ]; then A="--surface ddp"; E=""; else A=""; E="GRACE_WGRAD_STREAM=0"; fi
  cd /tmp && env $E timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/$v -o run -- \
    python3 $R/bench.py --steps 10 --warmup 5 $A > $D/$v.log 2>&1 || exit 1
  cd $R && python3 tools/prof_summary.py $D/$v/run_kernel_trace.csv --steps 8 --marker topk2_split --per-step-markers 1 \
    --top 60 > $D/sum_$v.txt && rm -f $D/$v/run_kernel_trace.csv || exit 1
  echo "== $v"; grep -o '"value": [0-9.]*' $D/$v.log; head -3 $D/sum_$v.txt
done
