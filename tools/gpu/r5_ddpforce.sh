#!/bin/bash
# Pin each conv3x3 backend / conv->BN choice for every layer in turn and compare the plain-DDP
# gradients (stream off, then on, as the test) against the fp64 CPU reference.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; mkdir -p gpurun_out/ddpforce
out=gpurun_out/ddpforce/force.jsonl; : > $out
for f in dgrad=miopen dgrad=mfma dgrad=mfma_t1 dgrad=mfma_t2 dgrad=mfma_t3 dgrad=mfma_t4 \
         fwd=miopen fwd=mfma fwd=mfma_t1 fwd=mfma_t2 fwd=mfma_t3 fwd=mfma_t4 \
         wgrad=miopen wgrad=mfma wgrad=mfma_t1 wgrad=mfma_t2 wgrad=mfma_t3 wgrad=mfma_t4 \
         bn=unfused bn=stats_t1 bn=stats_t2 bn=stats_t3 bn=stats_t4; do
  timeout -k 10 100 python -u tools/gpu/ddp_fp64_diag.py --tag $f --force $f --modes ddp_off,ddp_on,ddp_on_poison >> $out 2>gpurun_out/ddpforce/err_$f.log
  rc=$?
  echo "$f rc=$rc $(grep -o '"max_param_rel_err": [0-9.e+-]*' $out | tail -3 | tr '\n' ' ')"
  [ $rc -eq 0 ] || exit 1
done
GRACE_CONV3X3=0 timeout -k 10 100 python -u tools/gpu/ddp_fp64_diag.py --tag c3off >> $out 2>gpurun_out/ddpforce/err_c3off.log
echo "c3off rc=$? $(grep -o '"max_param_rel_err": [0-9.e+-]*' $out | tail -6 | tr '\n' ' ')"
