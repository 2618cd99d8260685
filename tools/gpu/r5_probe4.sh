#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=gpurun_out/probe4; mkdir -p $D
for i in 1 2; do
timeout -k 10 120 python -u tools/gpu/bn_bwd_capture.py --force dgrad=mfma_t2 --variant pinned --modes ddp_off,plain_on,plain_off > $D/pinned$i.json 2> $D/pinned$i.err
rc=$?; echo "pinned rc=$rc"; python -c "
import json
for l in open('$D/pinned$i.json'):
    if not l.startswith('{'): continue
    d=json.loads(l); print(d['mode'], d['bn2_bias_rel_err'])
    for k in sorted(d):
        if k.startswith('dgrad'): print('  ',k, d[k])
        if k.startswith('bwd'): print('  ',k, {q: d[k][q] for q in ("db_vs_fp64","dy_sum_vs_fp64","db_rel","mask_vs_fp64_layer3.0","mask_vs_fp64_layer3.1","fwd_y_vs_fp64") if q in d[k]})
"; [ $rc -eq 0 ] || exit 1
done
timeout -k 10 200 python -u -m pytest tests/test_gpu_a_comm.py -x -q --timeout 150 --timeout-method thread -k "rccl_cta or native_rccl" > $D/rccl.log 2>&1
echo "rccl tests rc=$?"; tail -3 $D/rccl.log
