# PMC + kernel-trace breakdown over setups (tools/pmc_breakdown.py); run on the GPU box.
# Usage: S=c2:4:path64,c2:0:path64 EXTRA="--compact 0" TAG=x bash tools/pmcb_session.sh
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=${TAG:-pmcb}; O=gpurun_out/$TAG; mkdir -p $O
S=${S:-c2:4:path64,c2:0:path64,s8w0:0:path64,s0w4:0:path64,s0w0:0:path64}
EXTRA=${EXTRA:-}
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $O/p1 -o p1 -- python3 tools/pmc_breakdown.py --setups $S $EXTRA > $O/order.json 2> $O/p1.err && echo p1 ok && \
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 tools/pmc_breakdown.py --setups $S --launches 5 $EXTRA > $O/order_kt.json 2> $O/kt.err && echo kt ok
