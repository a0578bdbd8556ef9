#!/usr/bin/env bash
# Collect the profiles committed under profiles/<round>/ (run on the GPU box via gpurun):
#   1. rocprofv3 --kernel-trace --stats of the default bench command (kernel durations)
#   2. PMC passes (each its own run, --kernel-trace only): FETCH_SIZE, WRITE_SIZE, and the
#      SQ instruction mix, for the bench workload at each precision
# Usage: ROUND=r01 bash tools/make_profiles.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ROUND=${ROUND:-r01}; OUT=gpurun_out/prof_$ROUND
CONFIGS=${CONFIGS:-c2}; PRECS=${PRECS:-path64 f64 f32}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bench" -o bench -- \
    python3 bench.py --steps 200 --warmup 40 --no-cpu-baseline --no-sweep > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { echo "bench trace failed"; exit 1; }
echo "bench trace ok"
# the same bench with one frame at a time (every dispatch serial: rocprof's average is then
# directly the bench's one-stream kernel_ms) and the driver's default command
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bench_fif1" -o bench -- \
    python3 bench.py --steps 200 --warmup 40 --no-cpu-baseline --no-sweep --frames-in-flight 1 \
    > "$OUT/bench_fif1.json" 2> "$OUT/bench_fif1.err" || { echo "fif1 trace failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bench_default" -o bench -- \
    python3 bench.py --steps 20 --warmup 5 > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" \
    || { echo "default trace failed"; exit 1; }
echo "fif1 + default traces ok"
for cfg in $CONFIGS; do
  for prec in $PRECS; do
    for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"; do
      tag=$(echo "$grp" | awk '{print $1}')
      timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/pmc_${cfg}_${prec}_${tag}" -o pmc -- \
          python3 tools/kernel_runner.py --config "$cfg" --precision "$prec" --launches 5 \
          > "$OUT/pmc_${cfg}_${prec}_${tag}.log" 2>&1 || { echo "pmc $cfg $prec $tag failed"; exit 1; }
    done
    echo "pmc $cfg $prec ok"
  done
done
