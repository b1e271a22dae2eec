#!/usr/bin/env python3
# SPDX-License-Identifier: GPL-2.0
"""Diagnostic (not a test): the RX launch over a pool of 2 M frames laid
down R times back to back in HBM (bench.py side_run's replicate), R = 1, 2,
4, 8 (or argv), to separate per-frame cost from pool size (address-
translation reach, clock): ms per launch and per 2 M frames, verdicts
checked.

    python tools/rep_probe.py [size] [R,R,...] [steps]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "bpf-examples_amd"))
import torch  # noqa: E402
import xdpgpu  # noqa: E402

size = int(sys.argv[1]) if len(sys.argv) > 1 else 1500
reps = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,2,4,8").split(",")]
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
n = 2 << 20
dev = torch.device("cuda:0")
u, ds, ex = xdpgpu.pool_generate(n, xdpgpu.POOL_UDP4, size, 0x5EED0012)
ctx = xdpgpu.XdpGpu(0, xdpgpu.CFG_DEFAULT, 0, xdpgpu.TUPLE_V4, 64)
for r in reps:
    g = torch.empty(u.nbytes * r + 64, dtype=torch.uint8, device=dev)
    src = torch.from_numpy(u).to(dev)
    for k in range(r):
        g[k * u.nbytes:(k + 1) * u.nbytes].copy_(src)
    del src
    rd = np.tile(ds, r)
    rd["addr"] += np.repeat(np.arange(r, dtype=np.uint64) * np.uint64(u.nbytes), n)
    gd = torch.from_numpy(rd.view(np.uint8).reshape(-1).copy()).to(dev)
    m = n * r
    gv = torch.empty(m, dtype=torch.uint8, device=dev)
    gr = torch.empty(m * 16, dtype=torch.uint8, device=dev)
    gt = torch.empty(m * 16, dtype=torch.uint8, device=dev)
    usize = g.numel() - 64
    for _ in range(3):
        ctx.process_dev(g, usize, gd, m, gv, gr, gt)
    ctx.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx.process_dev(g, usize, gd, m, gv, gr, gt)
    ctx.sync()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    ok = bool(np.array_equal(gv.cpu().numpy(), np.tile(ex, r)))
    print(json.dumps({"size": size, "replicas": r, "frames": m, "pool_gb": round(usize / 1e9, 2),
                      "ms_per_launch": round(ms, 4), "ms_per_2M": round(ms / r, 4),
                      "verdicts_ok": ok}), flush=True)
    del g, gd, gv, gr, gt
    torch.cuda.empty_cache()
