# GPU-box sanity pass: gpu tests, smoke, headline bench (each step bounded, chained with &&)
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 && tail -3 gpurun_out/gputests.log &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -2 gpurun_out/smoke.log &&
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log
