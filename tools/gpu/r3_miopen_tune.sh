#!/bin/bash
# Round 3: does an exhaustive MIOpen perf-db search (no gfx950 perf db ships with ROCm 7.2 or
# torch's bundled MIOpen, so every solver runs its default/heuristic config) speed up the fp32
# ResNet-50 convolutions?  baseline bench -> tuning pass into a repo-local user db -> bench again.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out/miopen_udb
(while sleep 50; do echo "tick $(date +%T) $(ls gpurun_out/miopen_udb | wc -l) files $(du -sk gpurun_out/miopen_udb | cut -f1) KB"; done) &
TICK=$!
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --exposed-steps 0 > gpurun_out/tune_base.log 2>&1 && grep '"metric"' gpurun_out/tune_base.log | cut -c1-200 &&
MIOPEN_USER_DB_PATH=$R/gpurun_out/miopen_udb MIOPEN_FIND_ENFORCE=SEARCH timeout -k 10 800 python bench.py --steps 2 --warmup 2 --exposed-steps 0 > gpurun_out/tune_search.log 2>&1; rc=$?
echo "search rc=$rc"; ls -la gpurun_out/miopen_udb
[ $rc -eq 0 ] || [ $rc -eq 124 ] || { kill $TICK; exit $rc; }
[ $rc -eq 124 ] && { kill $TICK; exit 124; }
MIOPEN_USER_DB_PATH=$R/gpurun_out/miopen_udb timeout -k 10 300 python bench.py --steps 30 --warmup 10 --exposed-steps 0 > gpurun_out/tune_after.log 2>&1 && grep '"metric"' gpurun_out/tune_after.log | cut -c1-200
rc=$?; kill $TICK; exit $rc
