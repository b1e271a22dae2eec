#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --pmc only) over the RX
# kernel on the config-2 pool (or PMC_CMD, e.g. tools/nat64_probe.py);
# summarised by tools/pmc_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=${OUT:-gpurun_out/pmc}
VARIANT=${VARIANT:-64:0}
DEST=${DEST:-}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS=${PMC_ARGS:-}
CMD=${PMC_CMD:-"python3 tools/tune_rx.py --variants $VARIANT --rounds 1 --reps 3 $ARGS"}
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
	   "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
	   "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
	i=$((i+1))
	echo "== pass $i: $grp"
	timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- $CMD > $OUT/p$i.log 2>&1
	rc=$?
	echo "== pass $i rc=$rc"
	if [ $rc -ne 0 ]; then tail -20 $OUT/p$i.log; exit $rc; fi
done
python3 tools/pmc_summary.py $OUT $DEST
