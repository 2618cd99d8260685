#!/bin/bash
# Whole-step graph with the GRACE exchange on a side stream (one fork/join per bucket) vs on the
# main stream, fp32 ResNet-50 Top-K, several bucket sizes.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
printf -- "%s\n" "--steps 30 --warmup 10 --overlap off" "--steps 30 --warmup 10 --overlap on" \
  "--steps 30 --warmup 10 --overlap on --bucket-mb 25" "--steps 30 --warmup 10 --overlap off --bucket-mb 128" \
  "--steps 30 --warmup 10 --overlap on --force-dist" "--steps 30 --warmup 10 --overlap off --force-dist" > gpurun_out/sweep_ov.txt
bash tools/bench_sweep.sh gpurun_out/sweep_ov.txt
