# depth-0 PMC passes for the F32 kernel (compare with tools/probe_depth.sh's PATH64 ones)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/probe
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/probe/f32pmc_d0 -o pmc -- python3 tools/kernel_runner.py --config c2 --precision f32 --launches 5 --depth 0 > gpurun_out/probe/f32pmc_d0.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/probe/f32pmc2_d0 -o pmc -- python3 tools/kernel_runner.py --config c2 --precision f32 --launches 5 --depth 0 > gpurun_out/probe/f32pmc2_d0.log 2>&1 || exit 1
