#!/usr/bin/env bash
# Host UBSan on the GPU paths (run on the GPU box through gpurun): the GPU test files against
# lib/ubsan/librt_amd.so (`make ubsan`: UndefinedBehaviorSanitizer on the C-ABI's host code,
# rt_capi.cpp and rt_multi.cpp — the multi-GPU exchange, the host pipeline — with the device
# code unchanged; the UBSan runtime is a dependency of the library, nothing is preloaded).
# Any report aborts the test process (-fno-sanitize-recover).  Build it beforehand, here, and
# take its line out of .gpurunignore for the run (it is listed there to keep pushes small).
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LIB=$PWD/ray-tracer-from-scratch_amd/lib/ubsan/librt_amd.so
[ -f "$LIB" ] || { echo "ubsan_gpu: build $LIB first (the ubsan target, here)"; exit 1; }
OUT=${OUT:-gpurun_out/ubsan}; mkdir -p "$OUT"
RT_AMD_LIB=$LIB UBSAN_OPTIONS=print_stacktrace=1:log_path=$OUT/ubsan \
    timeout -k 10 900 python -u -m pytest tests/test_multi_gpu.py tests/test_gpu_parity.py -x -q \
    --timeout 300 --timeout-method thread -m gpu > "$OUT/pytest.log" 2>&1 \
    || { echo "ubsan_gpu: tests failed (see $OUT)"; tail -5 "$OUT/pytest.log"; exit 1; }
ls "$OUT"/ubsan.* >/dev/null 2>&1 && { echo "ubsan_gpu: reports in $OUT"; exit 1; }
tail -1 "$OUT/pytest.log"
echo "ubsan_gpu: clean"
