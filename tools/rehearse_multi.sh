#!/usr/bin/env bash
# Rehearsal of bench.py's N-rank code paths on a one-GPU box: N ranks share the device
# (RT_BENCH_BACKEND=gloo; RCCL refuses two ranks on one GPU).  Checks that the frames mode
# and the tiled mode (uneven bands at N=3, RGBA8 transport) run end to end and print one
# JSON line; the numbers are not measurements.  Each run has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SESSION:-rehearse}
mkdir -p "$OUT"
export RT_BENCH_BACKEND=gloo
run() {  # name nproc args...
  local name=$1 n=$2; shift 2
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" \
      --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) \
      bench.py --gpus "$n" --steps 20 --warmup 5 --no-cpu-baseline $( [[ " $* " == *" --sweep-on "* ]] || echo --no-sweep ) ${@/--sweep-on/} \
      > "$OUT/$name.json" 2> "$OUT/$name.err"
  local rc=$?
  echo "$name rc=$rc: $(head -c 400 "$OUT/$name.json")"
  return $rc
}
# the tiled runs go through bench.py's N > 1 code (census all-reduce, torch tiler over gloo,
# steady state, the frame-sharded side run, max-over-ranks timing); tiled_n2_side keeps the
# side measurements on (no --no-sweep) so the frame-sharded side run is exercised too
run frames_n2 2 --mode frames && run tiled_n2 2 && run tiled_n3 3 \
  && run tiled_n3_rgba8 3 --out rgba8 && run tiled_n2_side 2 --sweep-on
