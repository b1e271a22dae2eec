# SPDX-License-Identifier: GPL-2.0
"""Host-registration probe (diagnostic, XDPGPU_HOSTREG_PROBE=1): logs, per
test, what the ROCm runtime holds registered over the host ranges the GPU
tests hand it -- the caller UMEMs xdpgpu_register_umem pins and maps, and
the pageable numpy sources of the tests' host-to-device copies (to_dev).

Every record is a JSON line in $XDPGPU_HOSTREG_OUT (default
gpurun_out/hostreg.jsonl).  hsa_amd_pointer_info only reads the runtime's
tables (tools/hostreg_probe.c), so the probe starts no GPU work."""
import ctypes as C
import json
import os

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
ENABLED = os.environ.get("XDPGPU_HOSTREG_PROBE") == "1"
OUT = os.environ.get("XDPGPU_HOSTREG_OUT", os.path.join(ROOT, "gpurun_out", "hostreg.jsonl"))
TYPES = {0: "unknown", 1: "hsa", 2: "locked", 3: "graphics", 4: "ipc", 5: "reserved",
         6: "vmem"}
PAGE = 4096

_lib = None
current_test = "?"
registered = []      # (base, size, test, closed)


def lib():
    global _lib
    if _lib is None:
        _lib = C.CDLL(os.path.join(ROOT, "tools", "libhostreg_probe.so"))
        _lib.hrp_scan.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_int]
        assert _lib.hrp_init() == 0
    return _lib


def scan(addr: int, size: int, max_rec: int = 64):
    """Runtime allocations covering [addr, addr + size)."""
    out = np.zeros(4 * max_rec, np.uint64)
    n = lib().hrp_scan(C.c_void_p(addr), size, C.c_void_p(out.ctypes.data), max_rec)
    assert n >= 0, "hsa_amd_pointer_info failed"
    return [{"type": TYPES.get(int(out[4 * k]), int(out[4 * k])),
             "host": hex(int(out[4 * k + 1])), "agent": hex(int(out[4 * k + 2])),
             "size": int(out[4 * k + 3])} for k in range(n)]


def log(event: str, **kw) -> None:
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with open(OUT, "a") as f:
        f.write(json.dumps({"test": current_test, "event": event, **kw}) + "\n")


def page_span(addr: int, size: int):
    lo = addr & ~(PAGE - 1)
    return lo, ((addr + size + PAGE - 1) & ~(PAGE - 1)) - lo


def install(xdpgpu, parity_module) -> None:
    """Wrap XdpGpu.register_umem / close and test_gpu_parity.to_dev."""
    orig_reg, orig_close = xdpgpu.XdpGpu.register_umem, xdpgpu.XdpGpu.close
    orig_to_dev = parity_module.to_dev

    def register_umem(self, umem, *a, **kw):
        base, size = umem.ctypes.data, umem.nbytes
        lo, sp = page_span(base, size)
        pre = scan(lo - PAGE, sp + 2 * PAGE)
        orig_reg(self, umem, *a, **kw)
        post = scan(lo - PAGE, sp + 2 * PAGE)
        log("register", base=hex(base), size=size, page_aligned=base % PAGE == 0,
            pre=pre, post=post)
        rec = [base, size, current_test, False]
        registered.append(rec)
        self._hostreg = getattr(self, "_hostreg", []) + [rec]

    def close(self):
        was_open = getattr(self, "h", None)
        orig_close(self)
        if not was_open:
            return
        for rec in getattr(self, "_hostreg", []):
            lo, sp = page_span(rec[0], rec[1])
            left = scan(lo, sp)
            rec[3] = True
            log("close", base=hex(rec[0]), size=rec[1], left=left)

    def to_dev(a, pad=64):
        base, size = a.ctypes.data, a.nbytes
        lo, sp = page_span(base, size)
        pre = scan(lo, sp)
        over = [r[:3] for r in registered if r[0] < base + size and base < r[0] + r[1]]
        t = orig_to_dev(a, pad)
        post = scan(lo, sp)
        if pre or post or over:
            log("to_dev", base=hex(base), size=size, pre=pre, post=post,
                overlaps_registered=[[hex(o[0]), o[1], o[2]] for o in over])
        return t

    xdpgpu.XdpGpu.register_umem = register_umem
    xdpgpu.XdpGpu.close = close
    parity_module.to_dev = to_dev


def end_of_test() -> None:
    """Any closed registration whose pages the runtime still holds."""
    for base, size, test, closed in registered:
        if not closed:
            continue
        lo, sp = page_span(base, size)
        left = scan(lo, sp)
        if left:
            log("stale", base=hex(base), size=size, registered_in=test, left=left)
