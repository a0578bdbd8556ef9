#!/usr/bin/env bash
# Host sanitizer check (CPU only): builds lib/asan/librt_amd.so (`make asan`: ASan + UBSan on
# the C-ABI's host code) and runs the CPU test files that drive that host code against it —
# scene packing, kernel-argument assembly, the pixel boxes and mirror chains over random
# scenes (test_bins_host), the boundary's argument checks (test_capi_host) and the C++
# drop-in (test_cpp_dropin).  Python itself is not instrumented, so the ASan runtime is
# preloaded and leak detection (which would report the interpreter's own allocations) is off.
set -eu
cd "$(dirname "$0")/.."
make -s -C ray-tracer-from-scratch_amd asan
ASAN_RT=$(/opt/rocm/bin/hipcc -print-file-name=libclang_rt.asan-x86_64.so)
for t in tests/test_bins_host.py tests/test_capi_host.py tests/test_cpp_dropin.py; do
  RT_AMD_LIB=$PWD/ray-tracer-from-scratch_amd/lib/asan/librt_amd.so LD_PRELOAD=$ASAN_RT \
  ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 \
      python -m pytest "$t" -q -p no:cacheprovider -m "not gpu" \
      || { echo "asan_check: $t failed (rerun with ASAN_OPTIONS/UBSAN_OPTIONS log_path=... for the report)"; exit 1; }
done
echo "asan_check: clean"
