#!/usr/bin/env python3
# SPDX-License-Identifier: GPL-2.0
"""Per-kernel summary of a rocprofv3 --kernel-trace database (rocpd SQLite),
in the shape of rocprofv3's kernel_stats.csv: name, calls, total/avg/min/max
duration (ns), percent, grid, VGPRs, LDS.  Usage:
    rocpd_stats.py RESULTS.db [--csv OUT.csv]"""
import argparse
import csv
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    rows = c.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration),"
        " max(duration), max(grid_x), max(vgpr_count), max(lds_size)"
        " from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    out = []
    for name, calls, tot, avg, mn, mx, grid, vgpr, lds in rows:
        out.append({"Name": name, "Calls": calls, "TotalDurationNs": int(tot),
                    "AverageNs": round(avg, 1), "MinNs": int(mn), "MaxNs": int(mx),
                    "Percentage": round(100.0 * tot / total, 2),
                    "GridX": grid, "VGPRs": vgpr, "LDS": lds})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    args = ap.parse_args()
    rows = stats(args.db)
    w = csv.DictWriter(open(args.csv, "w") if args.csv else sys.stdout,
                       fieldnames=list(rows[0].keys()) if rows else ["Name"])
    w.writeheader()
    for r in rows:
        w.writerow(r)
    if args.csv:
        for r in rows:
            print(f'{r["AverageNs"]/1e3:10.1f} us x{r["Calls"]:5d} {r["Percentage"]:6.2f}% '
                  f'vgpr {r["VGPRs"]:3d} grid {r["GridX"]:8d}  {r["Name"][:90]}')


if __name__ == "__main__":
    main()
