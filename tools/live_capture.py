#!/usr/bin/env python3
# SPDX-License-Identifier: GPL-2.0
"""Make tests/golden/live_capture.npz: frames received on a live AF_XDP
socket (copy mode, generic XDP redirect program, veth), as the RX ring
delivered them - chunk addresses and bytes - for tests/test_live.py.

The GPU box refuses AF_XDP (DESIGN.md "Live AF_XDP"), so the live receive
happens here (bpf-examples_amd/apps/xsk_probe --inject-file --capture) and
the GPU test replays the ring's descriptors over the captured UMEM.  The
frames sent are synthetic pools (xdpgpu.pool_generate, CPU): the xdpsock
shape, udp4 with its bad-checksum and malformed mixes, IMIX and ICMPv6
echo requests; frames the veth cannot carry (shorter than an Ethernet
header, longer than 1514 bytes) are left out."""
import os
import struct
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "bpf-examples_amd"))
import xdpgpu  # noqa: E402

PROBE = os.path.join(ROOT, "bpf-examples_amd", "apps", "xsk_probe")
OUT = os.path.join(ROOT, "tests", "golden", "live_capture.npz")


def pools():
    out = []
    for kind, size, n, seed, kw in ((xdpgpu.POOL_XDPSOCK, 64, 1024, 0x5EED0051, {}),
                                   (xdpgpu.POOL_UDP4, 64, 2048, 0x5EED0052, {}),
                                   (xdpgpu.POOL_IMIX, 64, 2048, 0x5EED0053, {}),
                                   (xdpgpu.POOL_UDP4, 128, 1024, 0x5EED0054,
                                    {"ppm_echo6": 300000})):
        u, d, _ = xdpgpu.pool_generate(n, kind, size, seed, **kw)
        eff = (d["addr"] & ((1 << 48) - 1)) + (d["addr"] >> 48)
        for k in range(n):
            ln = int(d["len"][k])
            if 14 <= ln <= 1514:
                out.append(bytes(u[int(eff[k]):int(eff[k]) + ln]))
    return out


def main():
    frames = pools()
    with tempfile.TemporaryDirectory() as td:
        inj = os.path.join(td, "inject.bin")
        cap = os.path.join(td, "capture.bin")
        with open(inj, "wb") as f:
            f.write(b"XGPI" + struct.pack("<I", len(frames)))
            for fr in frames:
                f.write(struct.pack("<I", len(fr)) + fr)
        r = subprocess.run([PROBE, "--inject-file", inj, "--capture", cap],
                           capture_output=True, text=True, timeout=120)
        print(r.stdout.strip())
        if r.returncode:
            sys.exit(f"xsk_probe failed ({r.returncode}): {r.stderr.strip()}")
        with open(cap, "rb") as f:
            blob = f.read()
    assert blob[:4] == b"XGPC"
    n, chunk = struct.unpack_from("<II", blob, 4)
    at = 12
    descs = np.zeros(n, xdpgpu.DESC_DTYPE)
    data = []
    for k in range(n):
        addr, ln, opt = struct.unpack_from("<QII", blob, at)
        at += 16
        descs[k] = (addr, ln, opt)
        data.append(blob[at:at + ln])
        at += ln
    assert at == len(blob) and n == len(frames)
    assert all(a == b for a, b in zip(data, frames)), "received bytes differ"
    lens = np.array([len(x) for x in data], np.uint32)
    np.savez_compressed(OUT, descs=descs.view(np.uint8), chunk=np.uint32(chunk),
                        lens=lens, frames=np.frombuffer(b"".join(data), np.uint8))
    print(f"wrote {OUT}: {n} frames, chunk {chunk}, "
          f"{len(np.unique(descs['addr'] // chunk))} distinct chunks")


if __name__ == "__main__":
    main()
