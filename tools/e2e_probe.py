#!/usr/bin/env python3
# SPDX-License-Identifier: GPL-2.0
"""The chunked host-path leg of bench.py alone (4 KiB chunks, 64 B frames
at headroom 256), with and without XDPGPU_CFG_UMEM_GATHER, and the host
time xdpgpu_submit takes per batch: for rocprofv3 (--kernel-trace
--memory-copy-trace --stats) and A/B runs.

    python3 tools/e2e_probe.py [--frames N] [--batches K] [--gather-only]

bench.py runs the gather leg through it as a child process: the gather is
the one kernel that reads host memory, and a fault there
then ends only the child, not the bench's line.
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


def submit_cost(cu, cd, B, flags, reps=8):
    """Host seconds per xdpgpu_submit call (the GPU work left queued)."""
    h = xdpgpu.XdpGpu(0, flags, 0, xdpgpu.TUPLE_V4, 0, max_batch=B)
    h.register_umem(cu, 4096)
    hd = xdpgpu.HostBuffer(B, xdpgpu.DESC_DTYPE)
    hd.array[:] = cd[:B]
    outs = [xdpgpu.HostBuffer(B, dt) for dt in (np.uint8, xdpgpu.RESULT_DTYPE,
                                                 xdpgpu.TUPLE4_DTYPE)]
    v, r, t = (b.array for b in outs)
    tot = 0.0
    for k in range(reps):
        t0 = time.perf_counter()
        h.submit(0, hd.array, v, r, t)
        tot += time.perf_counter() - t0
        h.wait(0)
    h.close()
    hd.close()
    for b in outs:
        b.close()
    return tot / reps


def e2e_queues(umem, descs, expect, queues: int, batches: int, B: int = 1 << 20,
               local: int = 0) -> dict:
    """Q RX queues on one GPU, as the reference runs one socket per queue:
    Q contexts on the same UMEM, each driven by its own thread (ctypes
    releases the GIL in the library), two batches in flight on each; the
    batches dealt round robin.  Aggregate frames / wall time."""
    import threading
    per = len(descs) // B
    ctxs, bufs = [], []
    for q in range(queues):
        h = xdpgpu.XdpGpu(local, xdpgpu.CFG_DEFAULT, 0, xdpgpu.TUPLE_V4, 0, max_batch=B)
        h.register_umem(umem, 0)
        hd = xdpgpu.HostBuffer(per * B, xdpgpu.DESC_DTYPE)
        hd.array[:] = descs[: per * B]
        outs = [[xdpgpu.HostBuffer(B, dt) for dt in (np.uint8, xdpgpu.RESULT_DTYPE,
                                                     xdpgpu.TUPLE4_DTYPE)] for _ in range(2)]
        ctxs.append(h)
        bufs.append((hd, outs))
    oks = [True] * queues

    def run(q, nb, check):
        h, (hd, outs) = ctxs[q], bufs[q]
        pending = [None, None]
        for k in range(nb + 2):
            slot = k & 1
            if pending[slot] is not None:
                h.wait(slot)
                if check:
                    lo = pending[slot]
                    oks[q] &= bool(np.array_equal(outs[slot][0].array, expect[lo:lo + B]))
                pending[slot] = None
            if k >= nb:
                continue
            lo = ((k * queues + q) % per) * B
            v, r, t = (b.array for b in outs[slot])
            h.submit(slot, hd.array[lo:lo + B], v, r, t)
            pending[slot] = lo

    def once(check):
        ths = [threading.Thread(target=run, args=(q, batches // queues, check))
               for q in range(queues)]
        t0 = time.perf_counter()
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        return time.perf_counter() - t0

    once(True)
    te = once(False)
    for h in ctxs:
        h.close()
    for hd, outs in bufs:
        hd.close()
        for o in outs:
            for b in o:
                b.close()
    fr = (batches // queues) * queues * B
    return {"queues": queues, "frames": fr, "batch": B, "mpps": round(fr / te / 1e6, 1),
            "h2d_gbps": round(fr * 80 / te / 1e9, 1), "d2h_gbps": round(fr * 33 / te / 1e9, 1),
            "verdicts_ok": all(oks)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1 << 20)
    ap.add_argument("--batches", type=int, default=32)
    ap.add_argument("--gather-only", action="store_true")
    ap.add_argument("--no-submit-cost", action="store_true")
    ap.add_argument("--compact", action="store_true",
                    help="XDPGPU_CFG_HOST_COMPACT on 4 KiB pages and on huge pages")
    ap.add_argument("--threads", default="0",
                    help="compaction thread counts to run (0: the library's default)")
    ap.add_argument("--h2d-ceil", type=float, default=57.0,
                    help="the box's pinned H2D GB/s (bench.py pcie_ceiling)")
    ap.add_argument("--d2h-ceil", type=float, default=57.0)
    ap.add_argument("--slots", default="2", help="batches in flight, e.g. 2,3,4")
    ap.add_argument("--queues", type=int, default=1,
                    help="RX queues: contexts, each driven by its own thread over its "
                         "share of the batches (packed leg)")
    ap.add_argument("--packed", action="store_true",
                    help="the packed leg instead (config-2 frames at a 64 B stride, "
                         "batches of 1 M, no chunk size)")
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    nc = args.frames
    if args.packed and args.queues > 1:
        cu, cd, ce = xdpgpu.pool_generate(nc, xdpgpu.POOL_UDP4, 64, 0x5EED0002)
        print(json.dumps(e2e_queues(cu, cd, ce, args.queues, args.batches)), flush=True)
        return
    if args.packed:
        cu, cd, ce = xdpgpu.pool_generate(nc, xdpgpu.POOL_UDP4, 64, 0x5EED0002)
        for slots in (int(x) for x in args.slots.split(",")):
            r = bench.e2e_run(0, cu, cd, ce, 1 << 20, args.batches, 0, 0,
                              {"h2d_gbps": args.h2d_ceil, "d2h_gbps": args.d2h_ceil},
                              xdpgpu.CFG_DEFAULT, slots)
            r.pop("pcie_ceiling", None)
            r["mode"] = "packed"
            h = xdpgpu.XdpGpu(0, xdpgpu.CFG_DEFAULT, 0, xdpgpu.TUPLE_V4, 0, max_batch=1 << 20)
            h.register_umem(cu, 0)
            hd = xdpgpu.HostBuffer(1 << 20, xdpgpu.DESC_DTYPE)
            hd.array[:] = cd[:1 << 20]
            outs = [xdpgpu.HostBuffer(1 << 20, dt) for dt in (np.uint8, xdpgpu.RESULT_DTYPE,
                                                             xdpgpu.TUPLE4_DTYPE)]
            v, rr, t = (b.array for b in outs)
            tot = 0.0
            for _ in range(8):
                t0 = time.perf_counter()
                h.submit(0, hd.array, v, rr, t)
                tot += time.perf_counter() - t0
                h.wait(0)
            h.close()
            r["submit_host_ms"] = round(tot / 8 * 1e3, 3)
            print(json.dumps(r), flush=True)
        return
    cu, cd, ce = xdpgpu.pool_generate(nc, xdpgpu.POOL_UDP4, 64, 0x5EED0032, stride=4096,
                                      headroom=256)
    ceil = {"h2d_gbps": args.h2d_ceil, "d2h_gbps": args.d2h_ceil}
    modes = [("gather", xdpgpu.CFG_DEFAULT | xdpgpu.CFG_UMEM_GATHER)]
    if not args.gather_only:
        modes.insert(0, ("rows", xdpgpu.CFG_DEFAULT))
    if args.compact:
        modes = [("compact", xdpgpu.CFG_DEFAULT | xdpgpu.CFG_HOST_COMPACT),
                 ("compact_huge", xdpgpu.CFG_DEFAULT | xdpgpu.CFG_HOST_COMPACT)]
    hu = bench.huge_pages_copy(cu) if args.compact else None
    runs = [(slots, name, flags, th) for slots in (int(x) for x in args.slots.split(","))
            for th in (int(x) for x in args.threads.split(","))
            for name, flags in modes if th == 0 or args.compact]
    for slots, name, flags, th in runs:
        if th:
            os.environ["XDPGPU_HOST_THREADS"] = str(th)
        else:
            os.environ.pop("XDPGPU_HOST_THREADS", None)
        u = hu if name.endswith("_huge") else cu
        r = bench.e2e_run(0, u, cd, ce, nc // 2, args.batches, 4096, 0, ceil, flags, slots)
        r.pop("pcie_ceiling", None)
        r["mode"] = name
        if not args.no_submit_cost:
            r["submit_host_ms"] = round(submit_cost(u, cd, nc // 2, flags) * 1e3, 3)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
