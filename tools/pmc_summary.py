#!/usr/bin/env python3
# SPDX-License-Identifier: GPL-2.0
"""Summarise rocprofv3 --pmc passes (tools/pmc_profile.sh) per kernel:
average counter value per dispatch.  HBM traffic per launch is
2 * FETCH_SIZE + WRITE_SIZE (KiB -> bytes): on gfx950 FETCH_SIZE reads half
the bytes of a wide coalesced stream (MI355X_MICROARCH.md §HBM).  PMC_ONLY:
sum only the kernels whose name holds it (default: the RX kernels)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


RX = ("xdp_rx_db_kernel", "xdp_rx_kernel", "xdp_rx_bulk_kernel", "xdp_rx_generic_kernel",
      "xdp_nat64_fast_kernel", "xdp_nat64_kernel")


def main(out, dest=None, frames=16 << 20, size=64, label=None):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get("Kernel_Name", "?")
                if ("xdp_" not in k and "synproxy" not in k and
                        not os.environ.get("PMC_ALL")):
                    continue
                name = row.get("Counter_Name")
                val = float(row.get("Counter_Value", 0))
                disp = row.get("Dispatch_Id")
                acc[k][name].append((disp, val))
    summary = {}
    for k, ctrs in acc.items():
        s = {}
        for name, vals in ctrs.items():
            per = defaultdict(float)
            for d, v in vals:
                per[d] += v
            s[name] = sum(per.values()) / max(len(per), 1)
        if "FETCH_SIZE" in s and "WRITE_SIZE" in s:
            s["hbm_bytes_per_launch"] = (2 * s["FETCH_SIZE"] + s["WRITE_SIZE"]) * 1024
        summary[k] = s
    print(json.dumps(summary, indent=1))
    with open(os.path.join(out, "summary.json"), "w") as fh:
        json.dump(summary, fh, indent=1)
    # bench.py form: HBM bytes per launch = sum over the launch's kernels
    only = os.environ.get("PMC_ONLY")
    rx = {k: v for k, v in summary.items()
          if (only in k if only else
              any(k.split("<")[0].split("(")[0].endswith(r) for r in RX))}
    tot = sum(v.get("hbm_bytes_per_launch", 0.0) for v in rx.values())
    doc = {"workload": label or (f"config2 pool: {frames} x {size} B IPv4/UDP "
                                 "(tools/tune_rx.py, V4 tuples)"),
           "frames": frames, "frame_size": size,
           "method": "rocprofv3 --pmc, one counter group per pass; "
                     "bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 "
                     "(gfx950 FETCH_SIZE halving, MI355X_MICROARCH.md HBM)",
           "hbm_bytes_per_launch": tot if rx else None,
           "per_kernel": summary}
    if dest:
        with open(dest, "w") as fh:
            json.dump(doc, fh, indent=1)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc",
         sys.argv[2] if len(sys.argv) > 2 else None,
         int(os.environ.get("FRAMES", 16 << 20)), int(os.environ.get("SIZE", 64)),
         os.environ.get("LABEL"))
