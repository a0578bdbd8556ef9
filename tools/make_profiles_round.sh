#!/usr/bin/env bash
# Per-round profiles (ROUND=rNN) (run on the GPU box via gpurun; every step has its own time limit):
#   1. rocprofv3 --kernel-trace --stats of the driver's bench command and of the one-stream
#      bench (frames in flight 1: rocprof's average dispatch = bench kernel_ms)
#   2. PMC passes, one counter group per pass, --kernel-trace only, on tools/kernel_runner.py:
#      FETCH_SIZE, WRITE_SIZE (HBM traffic), the SQ instruction mix, and the VALU activity
#      (SQ_ACTIVE_INST_VALU, SQ_THREAD_CYCLES_VALU, GRBM_GUI_ACTIVE) for c1, c2, c3, c5
# Then (here): python tools/summarize_profiles.py r03
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ROUND=${ROUND:?set ROUND=rNN}; OUT=gpurun_out/prof_$ROUND
CONFIGS=${CONFIGS:-c2 c1 c3 c5}; PRECS=${PRECS:-path64}
mkdir -p "$OUT"
if [ "${TRACES:-1}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bench_default" -o bench -- \
      python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" \
      || { echo "default trace failed"; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bench_fif1" -o bench -- \
      python3 bench.py --steps 200 --warmup 40 --no-cpu-baseline --no-sweep --frames-in-flight 1 \
      > "$OUT/bench_fif1.json" 2> "$OUT/bench_fif1.err" || { echo "fif1 trace failed"; exit 1; }
  echo "traces ok"
fi
for cfg in $CONFIGS; do
  for prec in $PRECS; do
    for grp in "FETCH_SIZE" "WRITE_SIZE" \
               "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" \
               "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
      tag=$(echo "$grp" | awk '{print $1}')
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/pmc_${cfg}_${prec}_${tag}" -o pmc -- \
          python3 tools/kernel_runner.py --config "$cfg" --precision "$prec" --launches 5 \
          > "$OUT/pmc_${cfg}_${prec}_${tag}.log" 2>&1 || { echo "pmc $cfg $prec $tag failed"; exit 1; }
    done
    echo "pmc $cfg $prec ok"
  done
done
exit 0
