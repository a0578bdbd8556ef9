#!/usr/bin/env bash
# Dispatch / cache PMC passes (SPI resource-allocation stalls, SQC instruction and scalar
# data caches) for one setup; two counters per pass, each pass its own run.
#   CFG=c2 PREC=path64 DEPTH=4 OUT=gpurun_out/pmcs bash tools/pmc_spi.sh
set -u
export TMPDIR=/tmp
CFG=${CFG:-c2}; PREC=${PREC:-path64}; DEPTH=${DEPTH:-4}; OUT=${OUT:-gpurun_out/pmcs}
mkdir -p "$OUT"
tag=${CFG}_${PREC}_d${DEPTH}
i=0
for grp in "SPI_RA_TGLIM_CU_FULL_CSN SPI_RA_WAVE_SIMD_FULL_CSN" "SPI_RA_VGPR_SIMD_FULL_CSN SPI_RA_REQ_NO_ALLOC_CSN" \
           "SQC_ICACHE_MISSES SQC_ICACHE_HITS" "SQC_DCACHE_MISSES SQC_DCACHE_HITS" "GRBM_GUI_ACTIVE GRBM_SPI_BUSY"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/${tag}_p$i" -o pmc -- \
      python3 tools/kernel_runner.py --config "$CFG" --precision "$PREC" --launches 5 --depth "$DEPTH" \
      > "$OUT/${tag}_p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/${tag}_p$i.log"; exit 1; }
done
echo "pmc_spi ok"
