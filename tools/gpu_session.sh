#!/bin/bash
# One gpurun session, steps named on the command line (in order):
#
#   bash tools/gpu_session.sh smoke pytest bench prof:config2 pmc ...
#
# Every step that touches the GPU runs under its own time limit.  Anything
# but exit 0 or a plain test/Python failure (1) ends the session at once
# (a fault, an abort, a time limit: nothing more runs on the GPU).  Each
# session writes into its own directory gpurun_out/<RUN>/ (RUN defaults to
# the UTC time), so a failing log is never overwritten by the next run.
#
# Steps:
#   smoke                  __graft_entry__.smoke()
#   pytest                 the whole -m gpu suite
#   pytest:FILE[,FILE..]   those test files only (-m gpu)
#   dbgtests:LIB:FILES     FILES (-m gpu) against a bounds-checked build
#                          (tests/conftest.py fails a test whose kernels
#                          clamped an access)
#   bench                  python bench.py (every leg)
#   bench:ARGS             python bench.py ARGS (words split on '+')
#   prof:NAME              rocprofv3 --kernel-trace --stats of a workload
#                          (config2 1500 imix imix_r2 nat64 nat64_egress
#                          nat64_dynamic frags synproxy echo)
#   pmc:NAME               PMC passes (tools/pmc_profile.sh) on a workload
#                          (config2 imix imix_r2 nat64 nat64_egress 1500)
#   ab:LIB                 A/B: the in-tree library vs LIB, alternating
#                          processes (IMIX, 1500 B, config 2)
#   abn:WL+WL:LIB,LIB      the same over named workloads and several LIBs
#   tune:WL:V,V            tune_rx variants (window:tune) interleaved in one
#                          process, 7 rounds, on a tune_rx workload
#   run:LIB:WORKLOAD       one workload (tune_rx timing) with library LIB
#   stamps[:N+TUNE+KIND+FMT] per-wave timeline (build/stamps, tools/stamps.py)
#   probe                  tools/order_probe (LDS-DMA / vmcnt ordering)
#   hbm[:MODE]             tools/hbm_probe [MODE] (access-shape ceilings)
#   e2e                    PCIe-inclusive host path (bench.py --e2e)
#   e2ec[:T,T]             host compaction legs (tools/e2e_probe.py --compact)
#   cli                    xdpsock-gpu over a 16 M-frame pool
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
RUN=${RUN:-$(date -u +%Y%m%dT%H%M%S)}
OUT=gpurun_out/$RUN
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== session $RUN: $*"

step() {  # name timeout cmd...
	local name=$1 t=$2; shift 2
	echo "== $name: $*"
	timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
	local rc=$?
	echo "== $name rc=$rc"
	tail -n 6 "$OUT/$name.log" | cut -c1-400
	if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
		echo "== stopping after $name (rc=$rc)"
		exit $rc
	fi
	return 0
}

# workload command lines shared by prof: and pmc:
workload() {
	case $1 in
	config2) echo "python3 tools/tune_rx.py --variants 64:0 --rounds 3" ;;
	1500) echo "python3 tools/tune_rx.py --variants 64:0 --rounds 3 --frames 2097152 --size 1500" ;;
	imix) echo "python3 tools/tune_rx.py --variants 64:0 --rounds 3 --frames 16777216 --kind 1 --seed 0x5EED0003 --fmt 2" ;;
	imix128) echo "python3 tools/tune_rx.py --variants 128:0 --rounds 3 --frames 16777216 --kind 1 --seed 0x5EED0003 --fmt 2" ;;
	1500_128) echo "python3 tools/tune_rx.py --variants 128:0 --rounds 3 --frames 2097152 --size 1500" ;;
	imix_r2) echo "python3 tools/tune_rx.py --variants 64:0 --rounds 3 --frames 16777216 --kind 1 --seed 0x5EED0003 --fmt 2 --ppm-v6 125000" ;;
	nat64) echo "python3 tools/nat64_probe.py --reps 5" ;;
	nat64_egress) echo "python3 tools/nat64_probe.py --reps 5 --direction 1" ;;
	nat64_dynamic) echo "python3 tools/nat_dyn_probe.py --frames 16777216 --reps 5" ;;
	frags) echo "python3 tools/frags_probe.py --reps 5" ;;
	frags_bounce) echo "python3 tools/frags_probe.py --reps 5 --tune 0x1000000" ;;
	synproxy) echo "python3 bench.py --no-cpu --no-e2e --legs synproxy --steps 5 --warmup 2" ;;
	echo) echo "python3 bench.py --no-cpu --no-e2e --legs echo --steps 5 --warmup 2" ;;
	echo_leg) echo "python3 tools/leg_probe.py --leg echo" ;;
	synproxy_leg) echo "python3 tools/leg_probe.py --leg synproxy" ;;
	bench) echo "python3 bench.py --no-cpu --no-secondary --no-e2e --steps 20" ;;
	bench50) echo "python3 bench.py --no-cpu --no-secondary --no-e2e --steps 50" ;;
	bench20) echo "python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-secondary --no-e2e" ;;
	*) echo "unknown workload $1" >&2; exit 2 ;;
	esac
}

for s in "$@"; do
	name=${s%%:*}
	arg=${s#*:}
	[ "$arg" = "$s" ] && arg=
	case $name in
	smoke) step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
	pytest)
		files=tests
		[ -n "$arg" ] && files=${arg//,/ }
		# shellcheck disable=SC2086
		step "pytest${arg:+_$(echo "$arg" | tr ',/' '__')}" 1100 python3 -u -m pytest $files \
			-m gpu -v --timeout 200 --timeout-method thread ;;
	dbgtests)
		lib=${arg%%:*}
		files=${arg#*:}
		# shellcheck disable=SC2086
		step "dbgtests_$(basename "$(dirname "$lib")")" 1100 env XDPGPU_LIB="$lib" \
			python3 -u -m pytest ${files//,/ } -m gpu -v --timeout 200 --timeout-method thread ;;
	bench)
		# shellcheck disable=SC2086
		step "bench${arg:+_$(echo "$arg" | tr '+-' '__')}" 600 python3 bench.py ${arg//+/ } ;;
	prof)
		# shellcheck disable=SC2046
		step "prof_$arg" 400 rocprofv3 --kernel-trace --stats --output-format csv \
			-d "$OUT/prof_$arg" -o run -- $(workload "$arg")
		f=$(find "$OUT/prof_$arg" -name '*kernel_trace.csv' | head -1)
		[ -n "$f" ] && python3 tools/trace_gaps.py "$f" --json "$OUT/prof_$arg/gaps.json" \
			> "$OUT/prof_$arg/gaps.txt" 2>&1
		true ;;
	pmc)
		# the pool's frame count and size for the summary (0: mixed sizes)
		case $arg in
		1500*) geo="FRAMES=2097152 SIZE=1500" ;;
		imix*) geo="FRAMES=16777216 SIZE=0" ;;
		nat64*) geo="FRAMES=16777216 SIZE=128" ;;
		echo_leg) geo="FRAMES=8388608 SIZE=128 PMC_ONLY=xdp_rx_db_kernel" ;;
		synproxy_leg) geo="FRAMES=8388608 SIZE=74 PMC_ONLY=synproxy_kernel" ;;
		*) geo="FRAMES=16777216 SIZE=64" ;;
		esac
		# shellcheck disable=SC2086
		step "pmc_$arg" 900 env $geo DEST="$OUT/pmc_$arg.json" OUT="$OUT/pmc_$arg" \
			PMC_CMD="$(workload "$arg")" LABEL="$arg" bash tools/pmc_profile.sh ;;
	pmcprobe)
		# PMC passes over tools/hbm_probe MODE, every kernel summarised
		# (the access-shape calibration of FETCH_SIZE / WRITE_SIZE)
		step "pmcprobe_$arg" 900 env PMC_ALL=1 DEST="$OUT/pmcprobe_$arg.json" \
			OUT="$OUT/pmcprobe_$arg" PMC_CMD="tools/hbm_probe $arg" LABEL="hbm_probe $arg" \
			bash tools/pmc_profile.sh ;;
	ab)
		for r in 1 2; do
			for lib in bpf-examples_amd/csrc/libxdpgpu.so "$arg"; do
				tag=$(basename "$(dirname "$lib")")_$r
				# shellcheck disable=SC2046
				step "ab_imix_$tag" 150 env XDPGPU_LIB="$lib" $(workload imix)
				# shellcheck disable=SC2046
				step "ab_1500_$tag" 150 env XDPGPU_LIB="$lib" $(workload 1500)
				# shellcheck disable=SC2046
				step "ab_config2_$tag" 150 env XDPGPU_LIB="$lib" $(workload config2)
			done
		done ;;
	abn)
		# abn:WL1+WL2:LIB1,LIB2 - two rounds, each workload, in-tree then each LIB
		wls=${arg%%:*}
		libs=${arg#*:}
		for r in 1 2; do
			for wl in ${wls//+/ }; do
				for lib in bpf-examples_amd/csrc/libxdpgpu.so ${libs//,/ }; do
					tag=$(basename "$(dirname "$lib")")_$r
					# shellcheck disable=SC2046
					step "abn_${wl}_$tag" 150 env XDPGPU_LIB="$lib" $(workload "$wl")
				done
			done
		done ;;
	tune)
		# tune:WL:V1,V2,... - tools/tune_rx.py variants (window:tune) in one
		# process, interleaved, on a tune_rx workload
		wl=${arg%%:*}
		vs=${arg#*:}
		# shellcheck disable=SC2046
		step "tune_${wl}_$(date +%s)" 300 $(workload "$wl" | sed "s/--variants 64:0/--variants $vs/; s/--rounds 3/--rounds 7/") ;;
	run)
		lib=${arg%%:*}
		wl=${arg#*:}
		# shellcheck disable=SC2046
		step "run_${wl}_$(basename "$(dirname "$lib")")_$(date +%s)" 200 env XDPGPU_LIB="$lib" \
			$(workload "$wl") ;;
	stamps)
		# shellcheck disable=SC2086
		step "stamps${arg:+_$(echo "$arg" | tr '+' '_')}" 200 env XDPGPU_LIB=build/stamps/libxdpgpu.so \
			python3 -u tools/stamps.py ${arg//+/ } ;;
	probe) step probe 120 tools/order_probe 64 ;;
	hbm) step "hbm_${arg:-all}" 300 tools/hbm_probe $arg ;;
	e2e) step e2e 600 python3 bench.py --no-cpu --no-secondary --steps 10 ;;
	e2ec)
		# the chunked host path with XDPGPU_CFG_HOST_COMPACT, 4 KiB and huge
		# pages, at the thread counts given (comma list, 0: the default)
		step "e2ec_${arg:-0}" 600 python3 tools/e2e_probe.py --compact --no-submit-cost \
			--threads "${arg:-0}" ;;
	cli) step cli 300 bpf-examples_amd/apps/xdpsock-gpu --pool 16777216 --pool-kind udp4 \
		-b 1048576 -C 67108864 --json -Q ;;
	*) echo "unknown step $s"; exit 2 ;;
	esac
done
echo "== session $RUN done"
