#!/bin/bash
# The driver's N = 1 bench command with the row order refreshed every 32 frames (default)
# vs measured once (1000000), interleaved; one JSON line per run into gpurun_out/abrf/.
set -o pipefail
mkdir -p gpurun_out/abrf
for rf in 32 1000000 1000000 32 32 1000000; do
  timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-sweep --no-cpu-baseline --no-c5 \
      --row-feedback $rf > gpurun_out/abrf/rf${rf}_$RANDOM.json 2>> gpurun_out/abrf/err.log || exit $?
done
