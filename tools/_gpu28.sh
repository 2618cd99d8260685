timeout -k 10 900 python -m pytest tests/test_gpu_engine.py -q -x > gpurun_out/t28.log 2>&1; echo T=$?; grep -E "passed|failed|Error" gpurun_out/t28.log | tail -5
cat > /tmp/s.txt <<'X'
--workload resnet50_topk --steps 50 --warmup 15 --grad-mode gather
--workload resnet50_topk --steps 50 --warmup 15 --grad-mode accumulate
--workload bert_qsgd --steps 30 --warmup 10 --grad-mode gather
--workload resnet50_none --steps 50 --warmup 15 --grad-mode gather
--workload vgg16_powersgd --steps 30 --warmup 10 --grad-mode gather
--workload lstm_efsignsgd --steps 30 --warmup 10 --grad-mode gather
X
bash tools/bench_sweep.sh /tmp/s.txt
