#!/usr/bin/env bash
# Build librt_amd.so with extra compile definitions into ray-tracer-from-scratch_amd/lib/ab/
# for in-process A/B (tools/ab.py).   Usage: tools/build_variant.sh NAME [-DX=1 ...]
set -eu
cd "$(dirname "$0")/../ray-tracer-from-scratch_amd"
name=$1; shift
B=build/ab_$name; mkdir -p "$B" lib/ab
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -munsafe-fp-atomics -I../include"
/opt/rocm/bin/hipcc $F "$@" -c csrc/rt_trace.hip -o "$B/rt_trace.o" &
/opt/rocm/bin/hipcc $F "$@" -c csrc/rt_trace_stamp.hip -o "$B/rt_trace_stamp.o" &
/opt/rocm/bin/hipcc $F "$@" -x hip -c csrc/rt_capi.cpp -o "$B/rt_capi.o" &
/opt/rocm/bin/hipcc $F "$@" -x hip -c csrc/rt_multi.cpp -o "$B/rt_multi.o" &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "lib/ab/$name.so" "$B/rt_trace.o" "$B/rt_trace_stamp.o" \
    "$B/rt_capi.o" "$B/rt_multi.o" -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "lib/ab/$name.so"
