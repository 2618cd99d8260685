#!/bin/bash
# Run bench.py once per "<args>" line and print one summary row per run (each under its own
# timeout; the first failure ends the sweep).  Lines come from a file ($1) or, with $1 = "--",
# from the remaining arguments.  Leading VAR=VALUE tokens are environment settings for that run.
#   bash tools/bench_sweep.sh sweep.txt
#   bash tools/bench_sweep.sh -- "--steps 30 --warmup 10" "--surface ddp --steps 30 --warmup 12"
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
T=${SWEEP_TIMEOUT:-300}
if [ "$1" = "--" ]; then shift; LINES=("$@"); else mapfile -t LINES < "$1"; fi
for v in "${LINES[@]}"; do
  [ -z "$v" ] && continue
  envs=(); args=()
  for t in $v; do if [ ${#args[@]} -eq 0 ] && [[ "$t" == *=* ]]; then envs+=("$t"); else args+=("$t"); fi; done
  env "${envs[@]}" timeout -k 10 "$T" python bench.py "${args[@]}" > gpurun_out/sweep_last.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "$v FAILED rc=$rc"; tail -8 gpurun_out/sweep_last.log; exit 1; fi
  grep '"metric"' gpurun_out/sweep_last.log | tail -1 | python3 -c "
import sys,json; d=json.loads(sys.stdin.read()); c=d['config']
print('$v', '|', d['value'], d['unit'], '|', d['ms_per_step'], 'ms | W', d['n_gpus'], 'seen', d.get('world_seen'),
      '|', c.get('hip_graph'), '| comm', c.get('comm'), '| host_issue', d.get('host_issue_ms_per_step'),
      '| grace_ms', d.get('grace_ms_per_step'), d.get('grace_ms_ci95', ''), '| per_rank', d.get('per_rank_ms_per_step'),
      '| rccl', d.get('rccl_nranks'), '| loss', d.get('final_loss'))"
done
