#!/bin/bash
# Round 4: exhaustive MIOpen perf-db search for the fp32 ResNet-50 b32 convolutions, resumable:
# the user db lives in gpurun_out/miopen_udb (merged back after each call, copied in before).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out/miopen_udb
[ -d tools/miopen_db ] && cp -n tools/miopen_db/* gpurun_out/miopen_udb/ 2>/dev/null
(while sleep 45; do echo "tick $(date +%T) $(ls gpurun_out/miopen_udb | wc -l) files $(du -sk gpurun_out/miopen_udb | cut -f1) KB" | tee -a gpurun_out/miopen_tick.log; done) &
TICK=$!
MIOPEN_USER_DB_PATH=$R/gpurun_out/miopen_udb MIOPEN_FIND_ENFORCE=SEARCH timeout -k 10 ${1:-1000} python bench.py --steps 2 --warmup 2 --exposed-steps 0 --grace-split off > gpurun_out/tune_search.log 2>&1; rc=$?
kill $TICK
echo "search rc=$rc"; ls -la gpurun_out/miopen_udb; tail -2 gpurun_out/tune_search.log | cut -c1-300
exit 0
