#!/bin/bash
# Round 4: A/B of the headline with the tuned MIOpen perf/find db (miopen_db/, produced by
# tools/gpu/r4_miopen_search.sh with MIOPEN_FIND_ENFORCE=SEARCH) against MIOpen's defaults.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
O=gpurun_out/r4_miopen_ab.txt; : > $O
for i in 1 2; do
  for cfg in tuned default; do
    rm -rf /tmp/mdb && mkdir -p /tmp/mdb
    [ $cfg = tuned ] && cp miopen_db/* /tmp/mdb/
    MIOPEN_USER_DB_PATH=/tmp/mdb timeout -k 10 300 python bench.py --steps 30 --warmup 10 --exposed-steps 0 --grace-split off > gpurun_out/r4_mab.log 2>&1 || { echo "FAILED $cfg"; tail -5 gpurun_out/r4_mab.log; exit 1; }
    echo "$cfg $(python3 tools/diag/benchline.py gpurun_out/r4_mab.log x)" | tee -a $O
  done
done
