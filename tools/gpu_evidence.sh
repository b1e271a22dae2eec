#!/bin/bash
# One gpurun session collecting the round's evidence: smoke, pytest -m gpu,
# bench.py (all legs), rocprofv3 --kernel-trace --stats per workload, PMC
# passes on config 2 and config 3 and the host-path / CLI rates.  Each GPU
# step has its own time limit; anything but exit 0 or a plain test failure
# (1) ends it.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name timeout cmd...
	local name=$1 t=$2; shift 2
	echo "== $name: $*"
	timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
	local rc=$?
	echo "== $name rc=$rc"
	tail -n 4 "$OUT/$name.log" | cut -c1-400
	if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
		echo "== stopping after $name (rc=$rc)"; exit $rc
	fi
}
prof() {  # name cmd...
	local name=$1; shift
	step "prof_$name" 300 rocprofv3 --kernel-trace --stats --output-format csv \
		-d "$OUT/prof_$name" -o run -- "$@"
}
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step pytest 900 python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread
step bench 600 python3 bench.py
prof config2 python3 bench.py --no-cpu --no-secondary --steps 20
prof 1500 python3 tools/tune_rx.py --variants 64:0 --rounds 3 --frames 2097152 --size 1500
prof imix python3 tools/tune_rx.py --variants 64:0 --rounds 3 --frames 16777216 --kind 1 --seed 0x5EED0003 --fmt 2
prof nat64 python3 tools/nat64_probe.py --reps 5
prof nat64_egress python3 tools/nat64_probe.py --reps 5 --direction 1
prof nat64_dynamic python3 tools/nat_dyn_probe.py --frames 16777216 --reps 5
prof frags python3 tools/frags_probe.py --reps 5
prof synproxy python3 bench.py --no-cpu --legs synproxy --steps 5 --warmup 2
step pmc 900 env DEST=$OUT/pmc_summary.json OUT=$OUT/pmc bash tools/pmc_profile.sh
step pmc_imix 900 env DEST=$OUT/pmc_imix_summary.json OUT=$OUT/pmc_imix LABEL="config3 pool: 16777216 IMIX frames, 44-byte network_tuple (tools/tune_rx.py)" PMC_ARGS="--frames 16777216 --kind 1 --seed 0x5EED0003 --fmt 2" bash tools/pmc_profile.sh
step e2e 600 python3 bench.py --no-cpu --no-secondary --steps 10 --e2e
step cli 300 bpf-examples_amd/apps/xdpsock-gpu --pool 16777216 --pool-kind udp4 -b 1048576 -C 67108864 --json -Q
