#!/usr/bin/env python3
# SPDX-License-Identifier: GPL-2.0
"""Diagnostic (not a test): the shader clock of one CU, sampled every
microsecond by tools/clock_probe.hip on a stream of its own, while the
config-2 RX launch runs back to back as bench.py times it (K launches on
the context's own stream).  Prints per-window effective clock (MHz) and,
under rocprofv3 --kernel-trace, the launches can be lined up with it.

    python tools/clock_trace.py [steps] [gap_us]

gap_us > 0 puts a host sleep of that many microseconds between launches
(the HIP-event pass's spacing), for comparison."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "bpf-examples_amd"))
import torch  # noqa: E402
import xdpgpu  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
gap_us = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
n = 16 << 20
probe = C.CDLL(os.path.join(ROOT, "tools", "libclock_probe.so"))
probe.clock_probe_launch.argtypes = [C.c_void_p, C.c_int, C.c_uint64, C.c_uint64, C.c_void_p]
umem, descs, expect = xdpgpu.pool_generate(n, xdpgpu.POOL_UDP4, 64, 0x5EED0002)
dev = torch.device("cuda:0")
d_umem = torch.zeros(umem.nbytes + 64, dtype=torch.uint8, device=dev)
d_umem[: umem.nbytes].copy_(torch.from_numpy(umem))
d_desc = torch.from_numpy(descs.view(np.uint8)).to(dev)
d_v = torch.empty(n, dtype=torch.uint8, device=dev)
d_res = torch.empty(n * 16, dtype=torch.uint8, device=dev)
d_tup = torch.empty(n * 16, dtype=torch.uint8, device=dev)
ctx = xdpgpu.XdpGpu(0, xdpgpu.CFG_DEFAULT, 0, xdpgpu.TUPLE_V4, 64)
for _ in range(5):
    ctx.process_dev(d_umem, umem.nbytes, d_desc, n, d_v, d_res, d_tup)
torch.cuda.synchronize()

maxs = 40000
buf = torch.zeros(2 * maxs + 1, dtype=torch.int64, device=dev)
side = torch.cuda.Stream(dev)
# sample for the expected run plus margin (100 MHz ticks), then stop
ticks = int((steps * (340 + gap_us) + 3000) * 100)
assert probe.clock_probe_launch(C.c_void_p(buf.data_ptr()), maxs, 100, ticks,
                                C.c_void_p(side.cuda_stream)) == 0
time.sleep(0.002)
t0 = time.perf_counter()
for _ in range(steps):
    ctx.process_dev(d_umem, umem.nbytes, d_desc, n, d_v, d_res, d_tup)
    if gap_us:
        torch.cuda.current_stream().synchronize()
        ctx.sync()
        time.sleep(gap_us * 1e-6)
ctx.sync()
t1 = time.perf_counter()
torch.cuda.synchronize()
b = buf.cpu().numpy().astype(np.uint64)
m = int(b[2 * maxs])
rt = b[0:2 * m:2].astype(np.float64)
ck = b[1:2 * m:2].astype(np.float64)
# effective clock per 20 us window
w = 20
mhz = []
for k in range(0, m - w, w):
    dr = (rt[k + w] - rt[k]) / 100.0          # us
    mhz.append(round((ck[k + w] - ck[k]) / dr, 1))
ok = bool(np.array_equal(d_v.cpu().numpy(), expect))
print(json.dumps({"steps": steps, "gap_us": gap_us, "samples": m,
                  "ms_per_step_host": round((t1 - t0) / steps * 1e3, 4),
                  "mhz_per_20us": mhz,
                  "mhz_pct": [round(float(x), 1) for x in np.percentile(mhz, [0, 10, 50, 90, 100])]
                  if mhz else None, "verdicts_ok": ok}))
