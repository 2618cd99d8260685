#!/bin/bash
# Run bench.py for each "<args>" line of $1 (one process each, 1 GPU) and print one summary row.
# Used on the GPU box: bash tools/bench_sweep.sh sweep.txt  (each run under its own timeout)
while IFS= read -r v; do
  [ -z "$v" ] && continue
  # leading VAR=VALUE tokens are environment settings for that run (e.g. GRACE_AMD_FORCE_TORCH=1)
  envs=(); args=()
  for t in $v; do if [ ${#args[@]} -eq 0 ] && [[ "$t" == *=* ]]; then envs+=("$t"); else args+=("$t"); fi; done
  env "${envs[@]}" timeout -k 10 300 python bench.py "${args[@]}" > gpurun_out/sweep_last.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "$v FAILED rc=$rc"; tail -5 gpurun_out/sweep_last.log; exit 1; fi
  grep '"metric"' gpurun_out/sweep_last.log | python3 -c "
import sys,json; d=json.loads(sys.stdin.read())
print('$v', '|', d['value'], d['unit'], '|', d['ms_per_step'], 'ms |', d['config'].get('hip_graph'), '| overlap', d['config'].get('overlap'), '| exposed', d.get('exposed_exchange_ms'), '| split', d.get('exchange_ms'), '| wire B', d.get('bytes_on_wire_per_rank'))"
done < "$1"
