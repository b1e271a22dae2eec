#!/usr/bin/env python3
# SPDX-License-Identifier: GPL-2.0
"""Diagnostic (not a test): GPU allocations of the HIP runtime that hold a
virtual range the CPU side of the process has NOT reserved, i.e. where a
later host mmap (a numpy array) can land and then be registered with
hipHostRegister, which maps host pages into the GPU at their own address.

Scans the holes between the process's CPU mappings (/proc/self/maps, the
mmap area) at 2 MiB steps with hsa_amd_pointer_info (tools/hostreg_probe.c:
table lookups only), before and after kernels that need scratch (private
segment) memory run: the runtime allocates a queue's scratch on first use.
Nothing here touches GPU memory from the host or launches a kernel on host
memory."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "bpf-examples_amd"))
import torch  # noqa: E402

import hostreg  # noqa: E402
import xdpgpu  # noqa: E402

STEP = 2 << 20


def maps():
    out = []
    with open("/proc/self/maps") as f:
        for line in f:
            p = line.split()
            lo, hi = (int(x, 16) for x in p[0].split("-"))
            out.append((lo, hi, p[1], p[5] if len(p) > 5 else ""))
    return sorted(out)


def gpu_outside_cpu_maps(cap=1 << 36):
    """HSA allocations whose first 2 MiB is not an accessible CPU mapping:
    scanned in the holes between mappings, below the lowest mapping of the
    mmap area (where new mmaps go, top-down) and inside PROT_NONE
    reservations, at most cap bytes of each."""
    m = [x for x in maps() if 0x700000000000 <= x[0] and x[1] < 0x7ff000000000]
    spans = [(m[0][0] - cap, m[0][0], "below")]
    for (a0, a1, _, _), (b0, _, _, _) in zip(m, m[1:]):
        if b0 > a1:
            spans.append((a1, min(b0, a1 + cap), "hole"))
    for a0, a1, perm, name in m:
        if perm.startswith("---"):
            spans.append((a0, min(a1, a0 + cap), "none:" + name))
    found, scanned = {}, 0
    cpu = [(a0, a1) for a0, a1, perm, _ in m if not perm.startswith("---")]
    for s0, s1, kind in spans:
        p = (s0 + STEP - 1) // STEP * STEP
        while p < s1:
            scanned += 1
            r = hostreg.scan(p, 1)
            if r:
                base = int(r[0]["host"], 16)
                found[base] = r[0] | {"where": kind, "cpu_accessible": any(
                    a0 <= base < a1 for a0, a1 in cpu)}
                p = max(p + STEP, (base + r[0]["size"] + STEP - 1) // STEP * STEP)
            else:
                p += STEP
    return list(found.values()), scanned


out = {}
dev = torch.device("cuda:0")
x = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
torch.cuda.synchronize()
out["after_torch_init"] = gpu_outside_cpu_maps()
# a kernel that needs scratch: nat64's general kernel (a /64 prefix takes
# it for every frame; 48-112 bytes of private memory a lane)
cfg, smap = xdpgpu.nat64_pool_config(xdpgpu.NAT64_INGRESS)
cfg.v6_plen = 64
u, d, _ = xdpgpu.pool_generate(4096, xdpgpu.POOL_NAT64, 128, 0x5EED0004)
du = torch.from_numpy(np.concatenate([u, np.zeros(64, np.uint8)])).to(dev)
dd = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
act = torch.empty(len(d), dtype=torch.uint8, device=dev)
od = torch.empty(len(d) * 16, dtype=torch.uint8, device=dev)
with xdpgpu.XdpGpu(0) as g:
    g.nat64_setup(cfg, smap)
    g.nat64_dev(du, u.nbytes, dd, len(d), act, od)
    g.sync()
torch.cuda.synchronize()
out["after_scratch_kernel"] = gpu_outside_cpu_maps()
out["maps"] = [(hex(a), hex(b), p, n) for a, b, p, n in maps() if a >= 0x700000000000]
print(json.dumps(out, indent=1))
