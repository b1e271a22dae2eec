#!/bin/bash
# Copy a tools/gpu_evidence.sh run (gpurun_out/) into profiles/ as round $1.
set -eu
R=${1:?round tag, e.g. r02}
O=gpurun_out
P=profiles
grep -h '^{"metric"' $O/bench.log | tail -1 > $P/${R}_bench.json
grep -h '^{"metric"' $O/e2e.log | tail -1 > $P/${R}_bench_e2e.json
grep -h '^{"prog"' $O/cli.log | tail -1 > $P/${R}_cli_xdpsock_gpu.json
tail -n 3 $O/pytest.log > $P/${R}_gpu_tests.txt
for w in config2 1500 imix nat64 nat64_egress nat64_dynamic frags synproxy; do
	f=$(ls $O/prof_$w/*kernel_stats.csv 2>/dev/null | head -1 || true)
	[ -n "$f" ] && cp "$f" $P/${R}_kernel_stats_$w.csv
done
cp $O/pmc_summary.json $P/${R}_pmc.json
cp $O/pmc_imix_summary.json $P/${R}_pmc_config3.json
ls -la $P | grep $R
