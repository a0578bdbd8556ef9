set -o pipefail
mkdir -p gpurun_out/abq
for n in 2 4; do
  for q in 4 16 16 4; do
    timeout -k 10 200 python3 bench.py --gpus $n --transport ipc --hw-queues $q --steps 20 --warmup 5 --no-sweep --no-cpu-baseline > gpurun_out/abq/n${n}_q${q}_$RANDOM.json 2>> gpurun_out/abq/err.log || exit $?
  done
done
