#!/usr/bin/env python3
# SPDX-License-Identifier: GPL-2.0
"""Diagnostic: per-kernel sums of rocprofv3 --pmc counter collections
(one directory per pass), averaged over dispatches."""
import collections
import csv
import glob
import sys

for d in sorted(glob.glob(sys.argv[1] + "/*/")):
    for f in glob.glob(d + "*counter_collection.csv"):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            per[(r["Kernel_Name"].split("(")[0], r["Counter_Name"], r["Dispatch_Id"])] += \
                float(r["Counter_Value"])
        agg = collections.defaultdict(list)
        for (k, c, _), v in per.items():
            agg[(k, c)].append(v)
        for (k, c), v in sorted(agg.items()):
            if sys.argv[2:] and not any(p in k for p in sys.argv[2:]):
                continue
            print(f"{k:60s} {c:16s} {sum(v) / len(v):16.0f}  n={len(v)}")
