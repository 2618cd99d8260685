#!/bin/bash
# DDP surface with batched library-wgrad copies: DDP tests, then bench --surface ddp on/off.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=$R/gpurun_out/ddpbatch; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_a_comm.py tests/test_gpu_wgrad.py -x -q --timeout 250 --timeout-method thread > $D/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|^E  " $D/tests.log | head -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/gpu/ddp_batch_debug.py 2>&1 | grep "^[0-9] " || exit 1
for v in 1 0 1 0; do
  GRACE_DDP_BATCH_COPY=$v timeout -k 10 300 python -u bench.py --surface ddp --steps 30 --warmup 10 > $D/b$v.json 2> $D/b$v.err || exit 1
  echo "batch=$v $(grep -o '"value": [0-9.]*' $D/b$v.json)"
done
timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $D/eng.json 2> $D/eng.err || exit 1
echo "engine $(grep -o '"value": [0-9.]*' $D/eng.json)"
