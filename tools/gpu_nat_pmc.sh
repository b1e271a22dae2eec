#!/bin/bash
# nat64 evidence: PMC passes on config 4 (ingress) and the egress pool.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
env DEST=$OUT/pmc_config4.json OUT=$OUT/pmc_nat LABEL="config4: 16777216 x 128 B IPv6 frames, nat64 ingress (tools/nat64_probe.py)" FRAMES=16777216 SIZE=128 PMC_CMD="python3 tools/nat64_probe.py --reps 3" bash tools/pmc_profile.sh > $OUT/pmc_nat.log 2>&1 || { tail -20 $OUT/pmc_nat.log; exit 1; }
env DEST=$OUT/pmc_nat64_egress.json OUT=$OUT/pmc_nateg LABEL="nat64 egress: 16777216 x 128 B IPv4 frames (tools/nat64_probe.py --direction 1)" FRAMES=16777216 SIZE=128 PMC_CMD="python3 tools/nat64_probe.py --reps 3 --direction 1" bash tools/pmc_profile.sh > $OUT/pmc_nateg.log 2>&1 || { tail -20 $OUT/pmc_nateg.log; exit 1; }
python3 - <<'PY'
import json
for f in ("gpurun_out/pmc_config4.json", "gpurun_out/pmc_nat64_egress.json"):
    d = json.load(open(f))
    print(f, d["hbm_bytes_per_launch"])
    for k, v in d["per_kernel"].items():
        print("  ", k[:60], {c: round(v.get(c, 0)) for c in ("FETCH_SIZE", "WRITE_SIZE", "hbm_bytes_per_launch", "TCC_HIT_sum", "TCC_MISS_sum")})
PY
