# A/B of environment settings on the headline bench (one process each)
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
run() { echo "== $*"; env "$@" timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/env_last.log 2>&1 || { tail -3 gpurun_out/env_last.log; return 1; }; grep '"metric"' gpurun_out/env_last.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['final_loss'])"; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_bnact.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_c1.log 2>&1; rc=$?; tail -2 gpurun_out/gpu_c1.log; [ $rc -eq 0 ] || exit $rc
run GRACE_AMD_CONV1X1=gemm && run GRACE_AMD_CONV1X1=conv && run GRACE_AMD_CONV1X1=gemm
