#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=gpurun_out/probe1; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_oob.py -x -q --timeout 250 --timeout-method thread > $D/oob.log 2>&1
rc=$?; echo "oob rc=$rc"; tail -4 $D/oob.log; [ $rc -le 1 ] || exit 1
timeout -k 10 120 python -u tools/gpu/bn_bwd_capture.py --force dgrad=mfma_t2 --variant pinned --modes ddp_off,plain_on,plain_off > $D/pinned.json 2> $D/pinned.err
rc=$?; echo "pinned rc=$rc"; cut -c1-900 $D/pinned.json; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u tools/gpu/bert_loss_trace.py --workload bert_none > $D/bert.json 2> $D/bert.err
rc=$?; echo "bert rc=$rc"; cut -c1-700 $D/bert.json
