#!/bin/bash
# Runs GPU steps in order, each under its own time limit: "LIMIT_SECONDS|command" per arg.
# A step that fails its tests (exit 1) does not stop the next; a time limit, abort or crash
# (124, 137, 134, 139, ...) ends the script there (nothing more runs on the GPU).
mkdir -p gpurun_out
worst=0
for spec in "$@"; do
  lim="${spec%%|*}"; cmd="${spec#*|}"
  echo "== step ($lim s): $cmd" >&2
  timeout -k 10 "$lim" bash -c "$cmd"
  rc=$?
  echo "== rc=$rc: $cmd" >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  [ $rc -gt $worst ] && worst=$rc
done
exit $worst
