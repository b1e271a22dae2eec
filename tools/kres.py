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


def code_objects(lib: str, arch: str = "gfx950") -> list:
    """The arch's code object of every offload bundle in the library (one
    per .hip translation unit)."""
    b = open(lib, "rb").read()
    objs = []
    i = b.find(b"__CLANG_OFFLOAD_BUNDLE__")
    while i >= 0:
        n = struct.unpack_from("<Q", b, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", b, p)
            p += 24
            triple = b[p:p + tl].decode()
            p += tl
            if triple.endswith(arch):
                objs.append(b[i + off:i + off + size])
        i = b.find(b"__CLANG_OFFLOAD_BUNDLE__", i + 24)
    if not objs:
        raise RuntimeError(f"{lib}: no {arch} code object")
    return objs


def kernels(lib: str = LIB) -> dict:
    out = ""
    for obj in code_objects(lib):
        with tempfile.NamedTemporaryFile(suffix=".elf") as f:
            f.write(obj)
            f.flush()
            out += subprocess.run([READELF, "--notes", f.name], capture_output=True,
                                  text=True, check=True).stdout
    res = {}
    # one record per kernel map (keys in alphabetical order: .args, whose
    # entries may carry .name too, come before the kernel's own .name)
    for blk in re.split(r"\n\s+- \.agpr_count:", out)[1:]:
        names = re.findall(r"\n    \.name:\s+(\S+)", blk)
        if not names:
            continue
        name = names[-1]

        def g(k):
            m = re.search(r"\n    \." + k + r":\s+(\d+)", blk)
            return int(m.group(1)) if m else None
        res[name] = {"vgpr": g("vgpr_count"), "sgpr": g("sgpr_count"),
                     "vgpr_spill": g("vgpr_spill_count"), "sgpr_spill": g("sgpr_spill_count"),
                     "scratch": g("private_segment_fixed_size"),
                     "lds": g("group_segment_fixed_size")}
    return res


if __name__ == "__main__":
    for k, v in kernels(sys.argv[1] if len(sys.argv) > 1 else LIB).items():
        print(json.dumps({"kernel": k, **v}))
