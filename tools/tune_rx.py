#!/usr/bin/env python3
# SPDX-License-Identifier: GPL-2.0
"""Interleaved A/B timing of RX kernel variants in one process (rules of
cdna_hip_programming.md §5.4 rule 24): the memory-ceiling kernel, and the
RX kernel per (window, tune).  Prints one JSON line per variant with the
median/min kernel time and algorithmic GB/s over ROUNDS rounds."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "bpf-examples_amd"))
import torch  # noqa: E402
import xdpgpu  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=16 << 20)
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--kind", type=int, default=xdpgpu.POOL_UDP4)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--seed", type=lambda x: int(x, 0), default=0x5EED0002)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--variants", default="ceil,64:0,64:256,64:512,128:0")
    ap.add_argument("--fmt", type=int, default=xdpgpu.TUPLE_V4)
    ap.add_argument("--ppm-v6", type=int, default=0,
                    help="IMIX: IPv6 frames per million (0: the pool's default)")
    args = ap.parse_args()
    n = args.frames
    kw = {"ppm_v6": args.ppm_v6} if args.ppm_v6 else {}
    umem, descs, expect = xdpgpu.pool_generate(n, args.kind, args.size, args.seed, **kw)
    dev = torch.device("cuda:0")
    d_umem = torch.zeros(umem.nbytes + 64, dtype=torch.uint8, device=dev)
    d_umem[: umem.nbytes].copy_(torch.from_numpy(umem))
    d_desc = torch.from_numpy(descs.view(np.uint8)).to(dev)
    d_v = torch.empty(n, dtype=torch.uint8, device=dev)
    d_res = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    tb = xdpgpu.TUPLE_BYTES[args.fmt]
    d_tup = torch.empty(max(1, n * tb), dtype=torch.uint8, device=dev)
    bpf = 16 + int(descs["len"].mean()) + 16 + tb + 1
    ctxs = {}
    for v in args.variants.split(","):
        if v == "ceil":
            ctxs[v] = xdpgpu.XdpGpu(0)
        else:
            w, t = (int(x, 0) for x in v.split(":"))
            ctxs[v] = xdpgpu.XdpGpu(0, xdpgpu.CFG_DEFAULT, 0, args.fmt, w, tune=t)
    s = torch.cuda.Stream(dev)
    times = {v: [] for v in ctxs}
    ok = {}
    for r in range(args.rounds):
        for v, ctx in ctxs.items():
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            fn = ctx.ceiling_dev if v == "ceil" else ctx.process_dev
            fn(d_umem, umem.nbytes, d_desc, n, d_v, d_res, d_tup, s)
            ev[0].record(s)
            for _ in range(args.reps):
                fn(d_umem, umem.nbytes, d_desc, n, d_v, d_res, d_tup, s)
            ev[1].record(s)
            torch.cuda.synchronize()
            times[v].append(ev[0].elapsed_time(ev[1]) / args.reps)
            if v != "ceil" and r == 0:
                ok[v] = bool(np.array_equal(d_v.cpu().numpy(), expect))
    splits = {}
    for v in ctxs:
        if v == "ceil":
            continue
        w, t = (int(x, 0) for x in v.split(":"))
        with xdpgpu.XdpGpu(0, xdpgpu.CFG_DEFAULT | xdpgpu.CFG_TIMING, 0, args.fmt, w,
                           tune=t) as tc:
            tc.process_dev(d_umem, umem.nbytes, d_desc, n, d_v, d_res, d_tup, s)
            torch.cuda.synchronize()
            tc.kernel_times()
            for _ in range(args.reps):
                tc.process_dev(d_umem, umem.nbytes, d_desc, n, d_v, d_res, d_tup, s)
            torch.cuda.synchronize()
            kt = tc.kernel_times()
            splits[v] = {k: round(kt[k], 4) for k in ("fast_ms", "exception_ms", "bulk_ms")}
    for v, ts in times.items():
        med = float(np.median(ts))
        print(json.dumps({"variant": v, "ms_median": round(med, 4),
                          "ms_min": round(min(ts), 4),
                          "gbps": round(n * bpf / med / 1e6, 1),
                          "gpps": round(n / med / 1e6, 2),
                          "frac": round(n * bpf / med / 1e6 / 8000, 4),
                          "verdicts_ok": ok.get(v), "split": splits.get(v)}), flush=True)


if __name__ == "__main__":
    main()
