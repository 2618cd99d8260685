R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1; rc=$?; tail -3 gpurun_out/gputests.log; [ $rc -eq 0 ] || exit $rc
printf -- "--workload bert_qsgd --steps 20 --warmup 10\n--workload bert_qsgd --steps 20 --warmup 10 --force-dist\n--steps 30 --warmup 10 --force-dist\n" > gpurun_out/sw9.txt && bash tools/bench_sweep.sh gpurun_out/sw9.txt
