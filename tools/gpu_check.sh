#!/bin/bash
# One gpurun session: smoke -> pytest -m gpu -> bench -> rocprofv3 stats
# -> PMC passes -> host-path (end-to-end) bench.
# Each GPU step has its own time limit; a crash/abort/timeout (anything but
# exit 0 or a plain Python failure 1) ends the session immediately.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out
mkdir -p $OUT
STEPS="${STEPS:-smoke pytest bench prof}"
step() {  # name timeout cmd...
	local name=$1 t=$2; shift 2
	echo "== $name: $*"
	timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
	local rc=$?
	echo "== $name rc=$rc"
	tail -n 25 "$OUT/$name.log"
	if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
		echo "== stopping after $name (rc=$rc)"; exit $rc
	fi
	return 0
}
for s in $STEPS; do
	case $s in
	smoke)  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
	pytest) step pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
	bench)  step bench 600 python bench.py ;;
	prof)   cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
		step prof 600 rocprofv3 --kernel-trace --stats --output-format csv \
			-d "$OUT/prof" -o run -- python3 bench.py --no-cpu --no-secondary --steps 20 ;;
	pmc)    step pmc 900 env DEST=$OUT/pmc_summary.json bash tools/pmc_profile.sh ;;
	e2e)    step e2e 600 python bench.py --no-cpu --no-secondary --steps 10 --e2e ;;
	esac
done
