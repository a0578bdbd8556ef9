#!/usr/bin/env bash
# Instruction-mix / issue PMC passes for one setup (each pass its own run, --kernel-trace only).
#   CFG=c2 PREC=path64 DEPTH=0 OUT=gpurun_out/pmcp bash tools/pmc_probe.sh
set -u
export TMPDIR=/tmp
CFG=${CFG:-c2}; PREC=${PREC:-path64}; DEPTH=${DEPTH:-0}; OUT=${OUT:-gpurun_out/pmcp}; LIB=${LIB:-}; OPT=${OPT:-}
mkdir -p "$OUT"
tag=${CFG}_${PREC}_d${DEPTH}${TAG:-}
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES" \
           "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_SENDMSG" \
           "SQ_INST_CYCLES_SALU SQ_INSTS_LDS SQ_INST_CYCLES_VMEM_RD SQ_IFETCH SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  [ -n "${PASSES:-}" ] && [ "${PASSES#*$i}" = "$PASSES" ] && continue
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/${tag}_p$i" -o pmc -- \
      python3 tools/kernel_runner.py --config "$CFG" --precision "$PREC" --launches 5 --depth "$DEPTH" ${LIB:+--lib $LIB} ${OPT:+--opt $OPT} \
      > "$OUT/${tag}_p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/${tag}_p$i.log"; }
done
