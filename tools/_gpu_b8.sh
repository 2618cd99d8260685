R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_mr.log 2>&1; rc=$?; tail -15 gpurun_out/gpu_mr.log; exit $rc
