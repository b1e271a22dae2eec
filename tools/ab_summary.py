#!/usr/bin/env python3
# SPDX-License-Identifier: GPL-2.0
"""Summarise a gpu_session.sh abn: run (gpurun_out/<RUN>/abn_<wl>_<lib>_<r>.log):
one line per workload and library with the measured figure of each round
(tune_rx: ms_median; bench legs: the leg's kernel ms)."""
import glob
import json
import os
import re
import sys
from collections import defaultdict


def figure(path):
    for line in reversed(open(path, errors="replace").read().splitlines()):
        line = line.strip()
        if not line.startswith("{"):
            continue
        try:
            j = json.loads(line)
        except ValueError:
            continue
        if "ms_median" in j:
            return j["ms_median"], j.get("verdicts_ok")
        for sec in j.values():
            if isinstance(sec, dict) and isinstance(sec.get("kernel_ms"), (int, float)):
                return sec["kernel_ms"], sec.get("verdicts_ok", True)
        if "ms_per_step" in j:
            return j["ms_per_step"], True
    return None, None


d = sys.argv[1]
res = defaultdict(dict)
for p in sorted(glob.glob(os.path.join(d, "abn_*.log"))):
    m = re.match(r"abn_([^_]+)_(.+)_(\d+)\.log$", os.path.basename(p))
    if m:
        res[m.group(1)].setdefault(m.group(2), []).append(figure(p))
for wl, libs in res.items():
    for lib, v in libs.items():
        print(f"{wl:8s} {lib:10s} " + "  ".join(f"{x}{'' if ok in (True, None) else ' BAD'}" for x, ok in v))
