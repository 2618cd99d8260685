#!/bin/bash
# Host-side AddressSanitizer preset: build the instrumented library and run the host checks.
set -e
R=$(cd "$(dirname "$0")/.." && pwd); cd "$R"
python -m grace_amd._build --asan
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
LD_PRELOAD="$RT" ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:detect_odr_violation=0 \
  GRACE_AMD_NATIVE_SO="$R/build/asan/_C.so" python tools/asan_host_check.py
