#!/usr/bin/env python3
# SPDX-License-Identifier: GPL-2.0
"""Diagnostic (not a test): the RX launch of a debug build (XDPGPU_LIB =
build/dbg/libxdpgpu.so, tools/dbg_build.sh) on the golden fixtures and a
small IMIX pool; prints the bounds-check record of xdpgpu_debug_read and
whether the verdicts match the fixtures / oracle."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "bpf-examples_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import torch  # noqa: E402
import xdpgpu  # noqa: E402
import oracle  # noqa: E402

lib = xdpgpu.load_library()
lib.xdpgpu_debug_read.argtypes = [C.c_void_p]
dbg = np.zeros(64, np.uint64)


def run(umem, descs, flags, iv, fmt, tune=0):
    n = len(descs)
    ctx = xdpgpu.XdpGpu(0, flags | xdpgpu.CFG_STATS, iv, fmt, 64, tune=tune)
    d_umem = torch.zeros(umem.nbytes + 64, dtype=torch.uint8, device="cuda:0")
    d_umem[: umem.nbytes].copy_(torch.from_numpy(umem))
    dd = np.ascontiguousarray(descs, xdpgpu.DESC_DTYPE).view(np.uint8)
    d_desc = torch.zeros(dd.nbytes + 16, dtype=torch.uint8, device="cuda:0")
    d_desc[: dd.nbytes].copy_(torch.from_numpy(dd))
    d_v = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda:0")
    d_res = torch.zeros(n * 16, dtype=torch.uint8, device="cuda:0")
    tb = xdpgpu.TUPLE_BYTES[fmt]
    d_tup = torch.zeros(max(n * tb, 1), dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    ctx.process_dev(d_umem, umem.nbytes, d_desc, n, d_v, d_res, d_tup)
    torch.cuda.synchronize()
    ctx.close()
    rc = lib.xdpgpu_debug_read(dbg.ctypes.data)
    rec = {int(k): [int(dbg[2 * k]), hex(int(dbg[2 * k + 1]))] for k in range(32) if dbg[2 * k]}
    return d_v.cpu().numpy(), rc, rec


fx = dict(np.load(os.path.join(ROOT, "tests", "golden", "fixtures.npz")))
meta = json.load(open(os.path.join(ROOT, "tests", "golden", "fixtures.json")))
descs = fx["descs"].view(xdpgpu.DESC_DTYPE)
for cfg in ("verify", "echo_net", "noverify"):
    flags, iv, fmt = meta["cfgs"][cfg]
    v, rc, rec = run(fx["umem"], descs, flags, iv, fmt)
    bad = np.nonzero(v != fx[f"{cfg}_verdict"])[0]
    print(f"golden {cfg}: rc {rc} checks {rec} verdict mismatches {len(bad)} {bad[:10].tolist()}",
          flush=True)
for name, kind, size, n in (("imix", xdpgpu.POOL_IMIX, 64, 100000),
                            ("udp64", xdpgpu.POOL_UDP4, 64, 1 << 20)):
    umem, d, expect = xdpgpu.pool_generate(n, kind, size, 0x5EED0003)
    for flags, fmt in ((0x5, 1), (0x5, 2)):
        v, rc, rec = run(umem, d, flags, 0, fmt)
        ov = oracle.process(umem.copy(), d, flags, 0, fmt)[0]
        print(f"{name} {flags:#x}/{fmt}: rc {rc} checks {rec} mismatches {(v != ov).sum()}",
              flush=True)
from test_max_frames import max_pool  # noqa: E402
umem, d, _ = max_pool()
for flags, iv, fmt in ((0x5, 0, 1), (0x7, 0x9E3779B9, 2), (0x4, 7, 1)):
    v, rc, rec = run(umem, d, flags, iv, fmt)
    ov = oracle.process(umem.copy(), d, flags, iv, fmt)[0]
    print(f"max {flags:#x}: rc {rc} checks {rec} mismatches {(v != ov).sum()}", flush=True)
