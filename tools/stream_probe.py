#!/usr/bin/env python3
# SPDX-License-Identifier: GPL-2.0
"""Diagnostic (not a test): tools/stream_probe.hip (one address-order pass
over a packed pool, producer and consumer waves, 61 output bytes a frame)
against the product's RX launch on the same config-3 IMIX pool, in one
process, alternating; the probe's per-frame sums checked on a sample.

    hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared \\
        -o tools/libstream_probe.so tools/stream_probe.hip
    python tools/stream_probe.py [--frames N] [--reps 5] [--rounds 3]"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "bpf-examples_amd"))
import torch  # noqa: E402
import xdpgpu  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=16 << 20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--kind", type=int, default=xdpgpu.POOL_IMIX)
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--lib", default="tools/libstream_probe.so",
                    help="the probe build (a variant) to time")
    a = ap.parse_args()
    lib = C.CDLL(os.path.join(ROOT, a.lib))
    lib.stream_probe.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32, C.c_void_p,
                                 C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
    n = a.frames
    umem, descs, expect = xdpgpu.pool_generate(n, a.kind, a.size, 0x5EED0003)
    eff = descs["addr"].astype(np.int64)
    assert (np.diff(eff) > 0).all(), "the probe needs descriptors in address order"
    dev = torch.device("cuda:0")
    d_umem = torch.zeros(umem.nbytes + 64, dtype=torch.uint8, device=dev)
    d_umem[: umem.nbytes].copy_(torch.from_numpy(umem))
    d_desc = torch.from_numpy(descs.view(np.uint8).reshape(-1)).to(dev)
    v = torch.empty(n, dtype=torch.uint8, device=dev)
    rec = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    tup = torch.empty(n * 44, dtype=torch.uint8, device=dev)
    ctr = torch.zeros(1, dtype=torch.int32, device=dev)
    blocks = torch.cuda.get_device_properties(0).multi_processor_count
    ctx = xdpgpu.XdpGpu(0, xdpgpu.CFG_DEFAULT, 0, xdpgpu.TUPLE_NET, 0)
    # one stream for both (not the null stream: handle 0 means the
    # context's own stream to the library)
    st = torch.cuda.Stream(dev)

    def probe():
        rc = lib.stream_probe(d_umem.data_ptr(), umem.nbytes, d_desc.data_ptr(), n,
                              v.data_ptr(), rec.data_ptr(), tup.data_ptr(), ctr.data_ptr(),
                              blocks, st.cuda_stream)
        assert rc == 0

    def product():
        ctx.process_dev(d_umem, umem.nbytes, d_desc, n, v, rec, tup, st.cuda_stream)

    def timed(fn):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(a.reps):
            fn()
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.reps

    res = {"probe_ms": [], "product_ms": []}
    for r in range(a.rounds):
        res["probe_ms"].append(round(timed(probe), 4))
        res["product_ms"].append(round(timed(product), 4))
        print(f"round {r}: probe {res['probe_ms'][-1]:.4f} ms, product "
              f"{res['product_ms'][-1]:.4f} ms", flush=True)
    ok_product = bool(np.array_equal(v.cpu().numpy(), expect))
    probe()
    torch.cuda.synchronize()
    # the probe's sums on a sample: 16-byte chunks over [eff & ~15,
    # round_up(eff + len, 16)), 16-bit halves added, folded
    rng = np.random.default_rng(1)
    idx = rng.choice(n, 4096, replace=False)
    r = rec.cpu().numpy().view(np.uint32).reshape(n, 4)
    bad = 0
    badv = []
    for i in idx:
        lo, hi = int(eff[i]) & ~15, (int(eff[i]) + int(descs["len"][i]) + 15) & ~15
        s = int(umem[lo:hi].view("<u2").astype(np.uint64).sum())
        while s >> 16:
            s = (s & 0xFFFF) + (s >> 16)
        if r[i, 0] != s:
            bad += 1
            f0 = (int(i) // 2048) * 2048
            a0 = int(eff[f0]) & ~15
            badv.append({"i": int(i), "len": int(descs["len"][i]), "seg_pos": int(i) - f0,
                         "off": int(eff[i]) - a0, "win": (int(eff[i]) - a0) // 32768,
                         "in_win": (int(eff[i]) - a0) % 32768, "got": int(r[i, 0]), "want": s,
                         "rec": [int(x) for x in r[i, 1:]]})
    for b in badv[:12]:
        print("bad", b)
    algo = n * (16 + 16 + 44 + 1) + int(descs["len"].astype(np.int64).sum())
    out = {"lib": a.lib, "frames": n, "pool_bytes": int(umem.nbytes), "algorithmic_bytes": algo,
           "probe_ms_median": float(np.median(res["probe_ms"])),
           "product_ms_median": float(np.median(res["product_ms"])),
           "probe_frac": round(algo / (np.median(res["probe_ms"]) * 1e-3) / 8e12, 4),
           "product_frac": round(algo / (np.median(res["product_ms"]) * 1e-3) / 8e12, 4),
           "probe_sums_bad": bad, "product_verdicts_ok": ok_product, "runs": res}
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
