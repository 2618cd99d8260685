R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fused_sgd.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_sgd.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_sgd.log; [ $rc -eq 0 ] || exit $rc
printf -- "--steps 30 --warmup 10\n--steps 30 --warmup 10 --optimizer torch\n--workload resnet50_none --steps 30 --warmup 10\n--workload vgg16_powersgd --steps 20 --warmup 10\n--workload bert_qsgd --steps 20 --warmup 10\n--workload lstm_efsignsgd --steps 40 --warmup 10\n--workload resnet9_dawn --steps 30 --warmup 10\n--workload resnet18_cifar_none --steps 30 --warmup 10\n" > gpurun_out/sw6.txt &&
bash tools/bench_sweep.sh gpurun_out/sw6.txt
