#!/usr/bin/env python3
# SPDX-License-Identifier: GPL-2.0
"""Config 2's device-resident step on one context (one RX queue, one
stream: each launch waits for the one before) against Q contexts (Q RX
queues on one GPU, each context its own stream and outputs, batches dealt
round robin): whether consecutive launches overlap the previous one's end
(the persistent kernel's last CUs) and the gap between launches.

    python3 tools/overlap_probe.py [--frames N] [--steps K] [--queues Q]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bpf-examples_amd"))

import bench  # noqa: E402
import xdpgpu  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=16 << 20)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--queues", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=4)
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    n = args.frames
    umem, descs, expect = xdpgpu.pool_generate(n, xdpgpu.POOL_UDP4, 64, 0x5EED0002)
    d_umem = bench.to_dev(umem, dev)
    d_desc = bench.to_dev(descs, dev, 0)
    outs = []
    ctxs = []
    for q in range(args.queues):
        outs.append((torch.empty(n, dtype=torch.uint8, device=dev),
                     torch.empty(n * 16, dtype=torch.uint8, device=dev),
                     torch.empty(n * 16, dtype=torch.uint8, device=dev)))
        ctxs.append(xdpgpu.XdpGpu(0, xdpgpu.CFG_DEFAULT, 0, xdpgpu.TUPLE_V4, 0))

    def run(nq):
        for k in range(3):
            c = ctxs[k % nq]
            c.process_dev(d_umem, umem.nbytes, d_desc, n, *outs[k % nq], None)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(args.steps):
            c = ctxs[k % nq]
            c.process_dev(d_umem, umem.nbytes, d_desc, n, *outs[k % nq], None)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.steps * 1e3

    res = {"1": [], str(args.queues): []}
    for _ in range(args.rounds):
        res["1"].append(round(run(1), 4))
        res[str(args.queues)].append(round(run(args.queues), 4))
    ok = all(bool(np.array_equal(o[0].cpu().numpy(), expect)) for o in outs)
    print(json.dumps({"frames": n, "steps": args.steps, "ms_per_step": res,
                      "verdicts_ok": ok}), flush=True)


if __name__ == "__main__":
    main()
