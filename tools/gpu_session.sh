#!/usr/bin/env bash
# One GPU session on the MI355X box: smoke -> parity tests -> bench -> rocprofv3 kernel trace.
# Every GPU step has its own time limit; a crash / abort / timeout (exit >= 2 from pytest,
# anything non-zero elsewhere) ends the session — no retries.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SESSION:-s1}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*"; }

step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc

step pytest-gpu
timeout -k 10 ${PYTEST_TIMEOUT:-600} python -m pytest tests -q -m gpu ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 "$OUT/pytest_gpu.log"
[ $rc -le 1 ] || exit $rc

step bench
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"; tail -5 "$OUT/bench.err"
[ $rc -eq 0 ] || exit $rc

if [ "${SWEEP:-1}" = 1 ]; then
  step sweep
  timeout -k 10 300 python tools/sweep.py ${SWEEP_ARGS:-} > "$OUT/sweep.jsonl" 2> "$OUT/sweep.err"
  rc=$?; echo "sweep rc=$rc"; cat "$OUT/sweep.jsonl"
  if [ $rc -eq 0 ] && [ -n "${SWEEP2_ARGS:-}" ]; then
    timeout -k 10 300 python tools/sweep.py ${SWEEP2_ARGS} > "$OUT/sweep2.jsonl" 2>> "$OUT/sweep.err"
    rc=$?; echo "sweep2 rc=$rc"; cat "$OUT/sweep2.jsonl"
  fi
  [ $rc -eq 0 ] || exit $rc
fi

if [ "${PROFILE:-1}" = 1 ]; then
  step rocprof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
      python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
  rc=$?; echo "rocprof rc=$rc"; find "$OUT/prof" -name '*stats*' | head; tail -3 "$OUT/prof.err"
fi
exit 0
