#!/usr/bin/env python3
# SPDX-License-Identifier: GPL-2.0
"""Per-kernel resources of the gfx950 code object inside libxdpgpu.so: the
clang offload bundle is unpacked in Python and the AMDGPU metadata notes
read with llvm-readelf (VGPRs, SGPRs, spills, scratch bytes a lane, LDS).

    python tools/kres.py [path/to/libxdpgpu.so]
"""
import json
import os
import re
import struct
import subprocess
import sys
import tempfile

READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "bpf-examples_amd", "csrc", "libxdpgpu.so")


def code_object(lib: str, arch: str = "gfx950") -> bytes:
    b = open(lib, "rb").read()
    i = b.find(b"__CLANG_OFFLOAD_BUNDLE__")
    if i < 0:
        raise RuntimeError(f"{lib}: no offload bundle")
    n = struct.unpack_from("<Q", b, i + 24)[0]
    p = i + 32
    for _ in range(n):
        off, size, tl = struct.unpack_from("<QQQ", b, p)
        p += 24
        triple = b[p:p + tl].decode()
        p += tl
        if triple.endswith(arch):
            return b[i + off:i + off + size]
    raise RuntimeError(f"{lib}: no {arch} code object")


def kernels(lib: str = LIB) -> dict:
    with tempfile.NamedTemporaryFile(suffix=".elf") as f:
        f.write(code_object(lib))
        f.flush()
        out = subprocess.run([READELF, "--notes", f.name], capture_output=True, text=True,
                             check=True).stdout
    res = {}
    for blk in out.split(".name:")[1:]:
        name = blk.split()[0]

        def g(k):
            m = re.search(r"\." + k + r":\s+(\d+)", blk)
            return int(m.group(1)) if m else None
        res[name] = {"vgpr": g("vgpr_count"), "sgpr": g("sgpr_count"),
                     "vgpr_spill": g("vgpr_spill_count"), "sgpr_spill": g("sgpr_spill_count"),
                     "scratch": g("private_segment_fixed_size"),
                     "lds": g("group_segment_fixed_size")}
    return res


if __name__ == "__main__":
    for k, v in kernels(sys.argv[1] if len(sys.argv) > 1 else LIB).items():
        print(json.dumps({"kernel": k, **v}))
