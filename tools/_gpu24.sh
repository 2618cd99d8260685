R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/t24.log 2>&1; echo T=$?; grep -E "passed|failed|Error|assert" gpurun_out/t24.log | tail -15
printf -- "--workload vgg16_powersgd --steps 30 --warmup 10\n" > /tmp/sw.txt
bash tools/bench_sweep.sh /tmp/sw.txt
