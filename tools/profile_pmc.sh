#!/usr/bin/env bash
# rocprofv3 PMC passes (one counter group per pass, --kernel-trace only; never combined
# with sys/runtime tracing) on tools/kernel_runner.py.  Usage:
#   CONFIG=c2 PREC=f64 OUT=gpurun_out/pmc bash tools/profile_pmc.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CONFIG=${CONFIG:-c2}; PREC=${PREC:-mixed}; OUT=${OUT:-gpurun_out/pmc}
mkdir -p "$OUT"
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d "$OUT/$name" -o pmc -- \
      python3 tools/kernel_runner.py --config "$CONFIG" --precision "$PREC" --launches 5 \
      > "$OUT/$name.log" 2>&1
  local rc=$?; echo "pass $name rc=$rc"; return $rc
}
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH || exit $?
run sq2 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC || exit $?
run sq3 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 || true
run sq4 SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_VALU GRBM_GUI_ACTIVE GRBM_COUNT || true
run tcc_fetch FETCH_SIZE || true
run tcc_write WRITE_SIZE || true
exit 0
