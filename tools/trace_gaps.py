#!/usr/bin/env python3
# SPDX-License-Identifier: GPL-2.0
"""Diagnostic (not a test): per-launch durations and the idle between
consecutive launches of one kernel, from a rocprofv3 --kernel-trace CSV
(`*_kernel_trace.csv`).  Launches that overlap (two streams) show a
negative gap.

    trace_gaps.py TRACE.csv [--kernel xdp_rx_db_kernel] [--json OUT]"""
import argparse
import csv
import json
import sys


def launches(path, kernel):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name") or r.get("KernelName") or ""
            if kernel in name:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                             r.get("Queue_Id", r.get("Stream_Id", ""))))
    rows.sort()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default="xdp_rx_db_kernel")
    ap.add_argument("--json")
    ap.add_argument("--last", type=int, default=20,
                    help="summarise the last K launches (bench.py's timed steps)")
    a = ap.parse_args()
    rows = launches(a.trace, a.kernel)
    out = []
    for i, (s, e, q) in enumerate(rows):
        gap = (rows[i + 1][0] - e) / 1e3 if i + 1 < len(rows) else None
        out.append({"i": i, "start_us": round((s - rows[0][0]) / 1e3, 1),
                    "dur_us": round((e - s) / 1e3, 1),
                    "gap_us": None if gap is None else round(gap, 1), "queue": q})
        print(f"{i:3d} start {out[-1]['start_us']:10.1f} dur {out[-1]['dur_us']:7.1f} "
              f"gap {'' if gap is None else f'{gap:7.1f}'} q {q}")
    summ = {}
    if len(rows) >= a.last > 0:
        t = rows[-a.last:]
        span = (max(e for _, e, _ in t) - t[0][0]) / 1e3
        summ = {"launches": a.last, "span_us": round(span, 1),
                "span_us_per_launch": round(span / a.last, 2),
                "mean_dur_us": round(sum(e - s for s, e, _ in t) / a.last / 1e3, 2),
                "queues": sorted({q for _, _, q in t})}
        print(f"last {a.last}: span {span:.1f} us = {span / a.last:.2f} us a launch; "
              f"mean duration {summ['mean_dur_us']:.2f} us; queues {summ['queues']}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"launches": out, "last": summ}, f, indent=0)
    return 0


if __name__ == "__main__":
    sys.exit(main())
