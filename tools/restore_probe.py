#!/usr/bin/env python3
# SPDX-License-Identifier: GPL-2.0
"""The echo leg's launch (bench.py echo_run) timed three ways: right after
the device-to-device restore of the pool on the same stream (as bench.py
did), after a synchronize that ends the restore first, and after the
restore, a synchronize and a small kernel of its own, and after the
restore and a 512 MiB read (the restore's dirty lines evicted): how much of
the events' span is the kernel and how much the restore's aftermath.

    python3 tools/restore_probe.py [--frames N] [--steps K]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bpf-examples_amd"))

import bench  # noqa: E402
import xdpgpu  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=8 << 20)
    ap.add_argument("--steps", type=int, default=8)
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream(dev)
    n = args.frames
    u, ds, ex = xdpgpu.pool_generate(n, xdpgpu.POOL_UDP4, 128, 0x5EED0042, ppm_echo6=200000)
    pristine = bench.to_dev(u, dev)
    work = torch.empty_like(pristine)
    d_desc = bench.to_dev(ds, dev, 0)
    d_v = torch.empty(n, dtype=torch.uint8, device=dev)
    d_res = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    d_tup = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    small = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
    # 512 MiB read after the restore: the restore's dirty lines written back
    # (evicted by clean ones) before the timed launch
    flush = torch.ones(64 << 20, dtype=torch.int64, device=dev)
    out = {}
    with xdpgpu.XdpGpu(0, xdpgpu.CFG_DEFAULT | xdpgpu.CFG_ICMP6_ECHO, 0,
                       xdpgpu.TUPLE_V4, 0) as g:
        for rnd in range(2):
            for mode in ("same_stream", "sync", "sync_small_kernel", "flush_read"):
                ms = []
                for k in range(args.steps + 2):
                    with torch.cuda.stream(stream):
                        work.copy_(pristine, non_blocking=True)
                    if mode != "same_stream":
                        torch.cuda.synchronize()
                    if mode == "flush_read":
                        with torch.cuda.stream(stream):
                            small[:8].view(torch.int64)[0] = flush.sum()
                        torch.cuda.synchronize()
                    if mode == "sync_small_kernel":
                        with torch.cuda.stream(stream):
                            small.fill_(k & 0xff)
                        torch.cuda.synchronize()
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    g.process_dev(work, u.nbytes, d_desc, n, d_v, d_res, d_tup, stream)
                    e1.record(stream)
                    torch.cuda.synchronize()
                    if k >= 2:
                        ms.append(e0.elapsed_time(e1))
                out.setdefault(mode, []).append(round(float(np.mean(ms)), 4))
    print(json.dumps({"frames": n, "kernel_ms": out}), flush=True)


if __name__ == "__main__":
    main()
