#!/usr/bin/env python3
# SPDX-License-Identifier: GPL-2.0
"""Diagnostic: multi-buffer packets (XDPGPU_CFG_FRAGS) against the same
frames as single descriptors.  A pool of jumbo frames is described twice:
one descriptor per frame, and each frame cut in place into fragments of at
most --chunk bytes (XDP_PKT_CONTD on all but the last).  Times both device
paths with HIP events on one stream and checks that every fragment carries
its frame's verdict."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bpf-examples_amd"))
import torch  # noqa: E402
import xdpgpu  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1 << 18)
    ap.add_argument("--size", type=int, default=9000)
    ap.add_argument("--chunk", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--tune", type=lambda x: int(x, 0), default=0,
                    help="cfg.tune of the fragments' context (1<<24: bounce copy)")
    args = ap.parse_args()
    u, d, _ = xdpgpu.pool_generate(args.frames, xdpgpu.POOL_UDP4, args.size, 0x5EED0002)
    lens = d["len"].astype(np.int64)
    nf = (lens + args.chunk - 1) // args.chunk
    frame_of = np.repeat(np.arange(len(d)), nf)
    k = np.arange(len(frame_of)) - np.repeat(np.cumsum(nf) - nf, nf)
    fd = np.zeros(len(frame_of), xdpgpu.DESC_DTYPE)
    fd["addr"] = d["addr"][frame_of] + k * args.chunk
    fd["len"] = np.minimum(lens[frame_of] - k * args.chunk, args.chunk)
    fd["options"] = np.where(k < nf[frame_of] - 1, xdpgpu.PKT_CONTD, 0)
    dev = torch.device("cuda:0")
    d_umem = torch.zeros(u.nbytes + 64, dtype=torch.uint8, device=dev)
    d_umem[:u.nbytes].copy_(torch.from_numpy(u))
    s = torch.cuda.Stream(dev)
    out = {}
    for name, descs, flags in (("frames", d, 0x5), ("fragments", fd, 0x5 | xdpgpu.CFG_FRAGS)):
        n = len(descs)
        d_desc = torch.from_numpy(descs.view(np.uint8)).to(dev)
        d_v = torch.zeros(n, dtype=torch.uint8, device=dev)
        d_res = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
        with xdpgpu.XdpGpu(0, flags, tune=args.tune if flags & xdpgpu.CFG_FRAGS else 0) as g:
            ms = []
            for r in range(args.reps + 1):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                g.process_dev(d_umem, u.nbytes, d_desc, n, d_v, d_res, None, stream=s)
                e1.record(s)
                torch.cuda.synchronize()
                if r:
                    ms.append(e0.elapsed_time(e1))
        out[name] = (float(np.median(ms)), d_v.cpu().numpy())
    ok = bool(np.array_equal(out["fragments"][1], out["frames"][1][frame_of]))
    gb = lens.sum() / 1e9
    for name in ("frames", "fragments"):
        t = out[name][0]
        print(f"{name}: {t:.4f} ms  {args.frames / t / 1e3:.1f} Mpkt/s  {gb / t * 1e3:.0f} GB/s")
    print(f"descriptors {len(fd)} for {len(d)} packets; verdicts_ok={ok}")


if __name__ == "__main__":
    main()
