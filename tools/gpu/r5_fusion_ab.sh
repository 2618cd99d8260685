#!/bin/bash
# Headline A/B after the implicit-GEMM loader change: default (with the autotune report), the BN
# prologue / backward-epilogue fusions that pin convs to the MFMA GEMM.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=gpurun_out/fusion_ab; mkdir -p $D
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $D/$tag.json 2> $D/$tag.err
  local rc=$?
  echo "$tag rc=$rc $(grep -o '"value": [0-9.]*\|"grace_ms_per_step": [0-9.]*' $D/$tag.json | tr '\n' ' ')"
  return $rc
}
run default GRACE_AUTOTUNE_REPORT=1 || exit 1
grep -c "mfma" $D/default.err; grep "^conv (" $D/default.err | cut -c1-60
run prologue1 GRACE_BN_PROLOGUE=1 || exit 1
run prologue2 GRACE_BN_PROLOGUE=2 || exit 1
run bwdepi GRACE_BN_BWD_EPI=1 || exit 1
run default2 GRACE_X=1 || exit 1
