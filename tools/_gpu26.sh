timeout -k 10 300 python -c "import __graft_entry__ as g; g.build(); g.smoke(); print('SMOKE OK')" 2>&1 | tail -3
bash tools/bench_sweep.sh tools/_sw26.txt
