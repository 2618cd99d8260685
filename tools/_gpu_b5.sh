R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1; rc=$?; tail -3 gpurun_out/gputests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log &&
timeout -k 10 400 python examples/cifar10_dawn.py --engine --epochs 24 --log gpurun_out/dawn_logs.tsv > gpurun_out/dawn.log 2>&1; rc=$?; tail -3 gpurun_out/dawn.log; exit $rc
