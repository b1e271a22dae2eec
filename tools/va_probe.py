#!/usr/bin/env python3
# SPDX-License-Identifier: GPL-2.0
"""Diagnostic (not a test, starts no kernel on host memory): where the HIP
runtime places device allocations and registered host memory in the
process's virtual address space.

For torch device tensors: is their GPU virtual range also reserved in the
CPU address space (/proc/self/maps), so that no host mmap can land on it?
For a host buffer registered with hipHostRegister(Mapped): is the device
pointer (hipHostGetDevicePointer) the host address itself (one VA for CPU
and GPU), and what does hsa_amd_pointer_info report for both?"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

hip = C.CDLL("libamdhip64.so")
hip.hipHostRegister.argtypes = [C.c_void_p, C.c_size_t, C.c_uint]
hip.hipHostUnregister.argtypes = [C.c_void_p]
hip.hipHostGetDevicePointer.argtypes = [C.POINTER(C.c_void_p), C.c_void_p, C.c_uint]

import hostreg  # noqa: E402


def maps():
    out = []
    with open("/proc/self/maps") as f:
        for line in f:
            p = line.split()
            lo, hi = (int(x, 16) for x in p[0].split("-"))
            out.append((lo, hi, p[1], p[5] if len(p) > 5 else ""))
    return out


def covering(m, lo, hi):
    """the CPU mappings overlapping [lo, hi)"""
    return [(hex(a), hex(b), perm, name) for a, b, perm, name in m if a < hi and lo < b]


res = {}
dev = torch.device("cuda:0")
ts = [torch.empty(n, dtype=torch.uint8, device=dev) for n in (1 << 20, 66 << 20, 512 << 20)]
torch.cuda.synchronize()
m = maps()
res["device_tensors"] = []
for t in ts:
    p = t.data_ptr()
    res["device_tensors"].append({
        "ptr": hex(p), "bytes": t.numel(),
        "cpu_maps": covering(m, p, p + t.numel()),
        "hsa": hostreg.scan(p, 1)})
# a host buffer as the tests make them (numpy, malloc/mmap), registered
for nbytes in (2 << 20, 71 << 20):
    a = np.zeros(nbytes, np.uint8)
    hp = a.ctypes.data
    rc = hip.hipHostRegister(hp, nbytes, 1)     # hipHostRegisterMapped
    dp = C.c_void_p()
    rc2 = hip.hipHostGetDevicePointer(C.byref(dp), hp, 0)
    m = maps()
    rec = {"host": hex(hp), "bytes": nbytes, "register_rc": rc, "devptr_rc": rc2,
           "devptr": hex(dp.value or 0), "same_va": (dp.value or 0) == hp,
           "hsa_host": hostreg.scan(hp, 1),
           "hsa_dev": hostreg.scan(dp.value, 1) if dp.value else None,
           "cpu_maps_host": covering(m, hp, hp + nbytes)[:4]}
    if dp.value and dp.value != hp:
        rec["cpu_maps_devptr"] = covering(m, dp.value, dp.value + nbytes)[:4]
    rec["unregister_rc"] = hip.hipHostUnregister(hp)
    rec["hsa_host_after"] = hostreg.scan(hp, 1)
    res.setdefault("registered", []).append(rec)
print(json.dumps(res, indent=1))

# -- a device allocation freed back to the runtime: does its VA leave the
# process's maps and the runtime's table together?  (No kernel touches
# anything below; registration is driver bookkeeping.)
import mmap as _mm  # noqa: E402

libc = C.CDLL("libc.so.6", use_errno=True)
libc.mmap.restype = C.c_void_p
libc.mmap.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_int, C.c_long]
libc.munmap.argtypes = [C.c_void_p, C.c_size_t]
MAP_FIXED_NOREPLACE = 0x100000
freed = []
for nbytes in (66 << 20, 8 << 20):
    t = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    p = t.data_ptr()
    before = {"cpu_maps": covering(maps(), p, p + nbytes), "hsa": hostreg.scan(p, 1)}
    del t
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    torch.cuda.synchronize()
    after = {"cpu_maps": covering(maps(), p, p + nbytes), "hsa": hostreg.scan(p, 1)}
    rec = {"ptr": hex(p), "bytes": nbytes, "live": before, "after_free": after}
    # a host mapping at exactly that VA, if the CPU side is free
    q = libc.mmap(p, nbytes, 3, 0x22 | MAP_FIXED_NOREPLACE, -1, 0)   # RW, PRIVATE|ANON
    rec["host_mmap_at_freed_va"] = hex(q) if q and q != C.c_void_p(-1).value else \
        f"failed errno {C.get_errno()}"
    if q == p:
        rec["hsa_over_host_mapping"] = hostreg.scan(p, 1)
        rc = hip.hipHostRegister(p, nbytes, 1)
        dp = C.c_void_p()
        rc2 = hip.hipHostGetDevicePointer(C.byref(dp), p, 0)
        rec["register"] = {"rc": rc, "devptr_rc": rc2, "devptr": hex(dp.value or 0),
                           "hsa": hostreg.scan(p, 1)}
        rec["unregister_rc"] = hip.hipHostUnregister(p)
        rec["hsa_after_unregister"] = hostreg.scan(p, 1)
        libc.munmap(p, nbytes)
    t2 = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    rec["next_alloc_same_size"] = hex(t2.data_ptr())
    del t2
    freed.append(rec)
print(json.dumps({"freed_device_va": freed}, indent=1))
