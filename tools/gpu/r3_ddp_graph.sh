#!/bin/bash
# DDP comm-hook surface captured as a whole-step HIP graph vs eager vs the engine (1x MI355X)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python bench.py --surface ddp --graph full --steps 30 --warmup 12 > gpurun_out/ddp_full.log 2>&1 && \
timeout -k 10 300 python bench.py --surface ddp --steps 30 --warmup 10 > gpurun_out/ddp_eager.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/ddp_engine_ref.log 2>&1
rc=$?
for f in ddp_full ddp_eager ddp_engine_ref; do
  python - "$f" <<'PY'
import json, sys
f = sys.argv[1]
try:
    lines = [l for l in open(f"gpurun_out/{f}.log") if l.startswith("{")]
    d = json.loads(lines[-1])
    print(f, d["value"], d["ms_per_step"], d["config"]["hip_graph"], d["config"].get("surface"), d.get("host_issue_ms_per_step"), d.get("final_loss"))
except Exception as e:
    print(f, "no result", e)
PY
done
exit $rc
