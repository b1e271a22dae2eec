#!/usr/bin/env python3
# SPDX-License-Identifier: GPL-2.0
"""Diagnostic: time xdpgpu_nat64_dev on the config-4 pool (HIP events on
the launch stream), for rocprofv3 --pmc passes and kernel A/B runs."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bpf-examples_amd"))
import torch  # noqa: E402
import xdpgpu  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=16 << 20)
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--direction", type=int, default=xdpgpu.NAT64_INGRESS)
    ap.add_argument("--tune", type=lambda x: int(x, 0), default=0)
    ap.add_argument("--headroom", type=int, default=None)
    ap.add_argument("--stride", type=int, default=None)
    args = ap.parse_args()
    kind = xdpgpu.POOL_NAT64 if args.direction == xdpgpu.NAT64_INGRESS else xdpgpu.POOL_NAT64_V4
    cfg, smap = xdpgpu.nat64_pool_config(args.direction)
    kw = {k: v for k, v in (("headroom", args.headroom), ("stride", args.stride)) if v is not None}
    u, ds, ex = xdpgpu.pool_generate(args.frames, kind, args.size, 0x5EED0004, **kw)
    dev = torch.device("cuda:0")
    pristine = torch.empty(u.nbytes + 64, dtype=torch.uint8, device=dev)
    pristine[u.nbytes:].zero_()
    pristine[:u.nbytes].copy_(torch.from_numpy(u))
    work = torch.empty_like(pristine)
    d_desc = torch.from_numpy(ds.view(np.uint8)).to(dev)
    n = len(ds)
    d_act = torch.empty(n, dtype=torch.uint8, device=dev)
    d_out = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream(dev)   # a real stream: the events must see the launch
    ms = []
    with xdpgpu.XdpGpu(0, tune=args.tune) as g:
        g.nat64_setup(cfg, smap)
        for k in range(args.reps + 1):
            with torch.cuda.stream(s):
                work.copy_(pristine)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            g.nat64_dev(work, u.nbytes, d_desc, n, d_act, d_out, s)
            e1.record(s)
            torch.cuda.synchronize()
            if k:
                ms.append(e0.elapsed_time(e1))
    ok = bool(np.array_equal(d_act.cpu().numpy(), ex))
    t = float(np.mean(ms))
    print(f"nat64 tune={args.tune:#x} dir={args.direction} frames={n} size={args.size}: {t:.4f} ms/launch "
          f"{n / t / 1e3:.1f} Mpps {n * 149 / t / 1e6:.1f} GB/s(149 B/frame) actions_ok={ok}")


if __name__ == "__main__":
    main()
