#!/usr/bin/env python3
# SPDX-License-Identifier: GPL-2.0
"""Diagnostic (not a test): config 2 timed as bench.py times it, K launches
back to back on one context, three ways interleaved in one process:
  serial   xdpgpu_process_dev on the context's stream (round 5's bench)
  slots    xdpgpu_submit_dev alternating the two slots, one output set a slot
  gapped   serial with a host sleep between launches (the clock's response)
Per round: wall ms a step and the GPU span of the K launches (events at
the two ends only) a step.

    python tools/pipeline_probe.py [--rounds 5] [--steps 20]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "bpf-examples_amd"))
import torch  # noqa: E402
import xdpgpu  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--frames", type=int, default=16 << 20)
    ap.add_argument("--modes", default="serial,slots")
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--kind", type=int, default=0, help="0 UDP4, 1 IMIX")
    ap.add_argument("--fmt", type=int, default=1, help="tuple format (1 V4, 2 NET)")
    ap.add_argument("--window", type=int, default=64)
    ap.add_argument("--seed", type=lambda x: int(x, 0), default=0x5EED0002)
    ap.add_argument("--idle", type=float, default=0.0,
                    help="seconds of host sleep (GPU idle) before each run")
    ap.add_argument("--prewarm", type=int, default=0,
                    help="launches before each run's warmup (after the idle)")
    a = ap.parse_args()
    n = a.frames
    umem, descs, expect = xdpgpu.pool_generate(n, a.kind, a.size, a.seed)
    tb = xdpgpu.TUPLE_BYTES[a.fmt]
    dev = torch.device("cuda:0")
    d_umem = torch.zeros(umem.nbytes + 64, dtype=torch.uint8, device=dev)
    d_umem[: umem.nbytes].copy_(torch.from_numpy(umem))
    d_desc = torch.from_numpy(descs.view(np.uint8).reshape(-1)).to(dev)
    outs = [(torch.empty(n, dtype=torch.uint8, device=dev),
             torch.empty(n * 16, dtype=torch.uint8, device=dev),
             torch.empty(n * tb, dtype=torch.uint8, device=dev)) for _ in range(2)]
    ctx = xdpgpu.XdpGpu(0, xdpgpu.CFG_DEFAULT, 0, a.fmt, a.window)
    ss = [torch.cuda.ExternalStream(ctx.slot_stream(i), device=dev) for i in range(2)]

    def launch(mode, k):
        if mode == "slots":
            ctx.submit_dev(k & 1, d_umem, umem.nbytes, d_desc, n, *outs[k & 1])
        else:
            ctx.process_dev(d_umem, umem.nbytes, d_desc, n, *outs[0])
            if mode == "gapped":
                time.sleep(30e-6)

    def run(mode):
        if a.idle:
            time.sleep(a.idle)
        for k in range(a.prewarm):
            launch(mode, k)
        for k in range(5):
            launch(mode, k)
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        e0.record(ss[0])
        ss[1].wait_event(e0)
        t0 = time.perf_counter()
        for k in range(a.steps):
            launch(mode, k)
        for i in range(2):
            e1[i].record(ss[i])
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / a.steps * 1e3
        span = max(e0.elapsed_time(e) for e in e1) / a.steps
        return wall, span

    res = {m: [] for m in a.modes.split(",")}
    for r in range(a.rounds):
        for m in res:
            w, s = run(m)
            res[m].append((round(w, 4), round(s, 4)))
            print(f"round {r} {m:7s} wall {w:.4f} ms/step  span {s:.4f}", flush=True)
    ok = all(np.array_equal(o[0].cpu().numpy(), expect) for o in outs[: 2 if "slots" in res else 1])
    summ = {m: {"wall_ms_median": float(np.median([x[0] for x in v])),
                "span_ms_median": float(np.median([x[1] for x in v])), "runs": v}
            for m, v in res.items()}
    summ["verdicts_ok"] = ok
    print(json.dumps(summ))
    ctx.close()


if __name__ == "__main__":
    main()
