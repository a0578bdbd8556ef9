#!/usr/bin/env bash
# Round-3 GPU session: GPU tests (new ones first), then bench runs.  Every GPU step has its
# own time limit; a crash / abort / timeout ends the session (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${S:-r3}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*"; }
if [ -n "${TESTS:-}" ]; then
  step pytest $TESTS
  timeout -k 10 ${PT:-900} python -u -m pytest $TESTS -x -v -m gpu --timeout 150 --timeout-method thread ${K:+-k "$K"} > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" "$OUT/pytest.log" | tail -5
  [ $rc -eq 0 ] || { tail -40 "$OUT/pytest.log"; exit $rc; }
fi
i=0
for args in "${B1-}" "${B2-}" "${B3-}" "${B4-}"; do
  i=$((i+1))
  [ -n "$args" ] || continue
  [ "$args" = "default" ] && args=""
  step bench$i $args
  timeout -k 10 300 python -u bench.py $args > "$OUT/bench$i.json" 2> "$OUT/bench$i.err"
  rc=$?; echo "bench$i rc=$rc"; head -c 3000 "$OUT/bench$i.json"; echo; tail -5 "$OUT/bench$i.err"
  [ $rc -eq 0 ] || exit $rc
done
exit 0
