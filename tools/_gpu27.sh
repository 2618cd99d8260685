timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/t27.log 2>&1; echo T=$?; grep -E "passed|failed|Error" gpurun_out/t27.log | tail -5
printf -- "--workload resnet50_topk --steps 50 --warmup 15\n--workload resnet50_topk --steps 50 --warmup 15\n" > /tmp/s.txt
bash tools/bench_sweep.sh /tmp/s.txt
