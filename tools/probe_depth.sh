set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/probe
timeout -k 10 120 python tools/wave_times.py --lib ray-tracer-from-scratch_amd/lib/ab/wt.so --setups c2:0:path64,c2:1:path64,c2:4:path64 > gpurun_out/probe/wt.log 2>&1 || exit 1
for d in 0 4; do
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/probe/pmc_d$d -o pmc -- python3 tools/kernel_runner.py --config c2 --precision path64 --launches 5 --depth $d > gpurun_out/probe/pmc_d$d.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/probe/pmc2_d$d -o pmc -- python3 tools/kernel_runner.py --config c2 --precision path64 --launches 5 --depth $d > gpurun_out/probe/pmc2_d$d.log 2>&1 || exit 1
done
