#!/bin/bash
# the 1500 B leg: round 5's bench.py (tools/bench_r05.py) against this one,
# alternating processes on one box
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06_ab1500
mkdir -p $O
for r in 1 2; do
	for b in tools/bench_r05.py bench.py; do
		tag=$(basename $b .py)_$r
		timeout -k 10 200 python3 $b --no-cpu --no-e2e --legs 1500 --steps 10 --warmup 2 > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
		python3 -c "
import json,sys
d=json.loads([l for l in open('$O/$tag.log') if l.startswith('{')][0])
s=d['secondary_1500B']
print('$tag', d['ms_per_step'], s['ms_per_launch'], s['kernel_ms'])"
	done
done
