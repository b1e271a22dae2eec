#!/bin/bash
# PMC passes (tools/pmc_profile.sh) of the 1500 B and IMIX workloads with
# 128-byte windows (tune_rx variant 128:0), into gpurun_out/$RUN/.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
RUN=${RUN:-pmcw}
O=gpurun_out/$RUN
mkdir -p $O
FRAMES=2097152 SIZE=1500 DEST=$O/pmc_1500_w128.json OUT=$O/pmc_1500 LABEL=1500-w128 \
	PMC_CMD="python3 tools/tune_rx.py --variants 128:0 --rounds 3 --frames 2097152 --size 1500" \
	timeout -k 10 600 bash tools/pmc_profile.sh > $O/pmc_1500.log 2>&1 || exit $?
FRAMES=16777216 SIZE=0 DEST=$O/pmc_imix_w128.json OUT=$O/pmc_imix LABEL=imix-w128 \
	PMC_CMD="python3 tools/tune_rx.py --variants 128:0 --rounds 3 --frames 16777216 --kind 1 --seed 0x5EED0003 --fmt 2" \
	timeout -k 10 600 bash tools/pmc_profile.sh > $O/pmc_imix.log 2>&1
