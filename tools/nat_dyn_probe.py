#!/usr/bin/env python3
# SPDX-License-Identifier: GPL-2.0
"""Time xdpgpu_nat64_dev with dynamic state on the config-4 pool: the static
mappings (--nstatic), a v4 pool widened to 10.98.0.0/15, the pool's other
sources allocated from next_addr 1 by the first launches, then steady
state.  Prints every launch."""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "bpf-examples_amd"))
import xdpgpu  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--nstatic", type=int, default=65533)
    ap.add_argument("--clock", type=int, default=10**13,
                    help="batch clock (ns); 0: CLOCK_MONOTONIC")
    a = ap.parse_args()
    dev = "cuda:0"
    cfg, smap = xdpgpu.nat64_pool_config(xdpgpu.NAT64_INGRESS)
    u, ds, ex = xdpgpu.pool_generate(a.frames, xdpgpu.POOL_NAT64, 128, 0x5EED0004)
    print(f"pool {a.frames}", flush=True)
    pristine = torch.from_numpy(u).to(dev)
    work = torch.empty_like(pristine)
    d_desc = torch.from_numpy(ds.view(np.uint8)).to(dev)
    d_act = torch.empty(a.frames, dtype=torch.uint8, device=dev)
    d_out = torch.empty(a.frames * 16, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream()
    with xdpgpu.XdpGpu(0) as g:
        cfg.v4_prefix, cfg.v4_mask = 0x0A620000, 0xFFFE0000
        g.nat64_setup(cfg, smap[:a.nstatic])
        g.nat64_dynamic(7200 * 10**9, 1)
        for k in range(a.reps):
            if a.clock:
                g.nat64_clock(a.clock + k)
            work.copy_(pristine)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            g.nat64_dev(work, u.nbytes, d_desc, a.frames, d_act, d_out, stream)
            torch.cuda.synchronize()
            t = time.perf_counter() - t0
            ent, nxt, q = g.nat64_state()
            print(f"launch {k}: {t * 1e3:.3f} ms, entries {len(ent)}, next_addr {nxt}, "
                  f"queue {len(q)}", flush=True)
    exd = ex.copy()
    exd[exd == xdpgpu.NAT64_NO_STATE] = xdpgpu.TC_ACT_REDIRECT
    act = d_act.cpu().numpy()
    print("actions", {int(k): int(v) for k, v in zip(*np.unique(act, return_counts=True))},
          "ok" if np.array_equal(act, exd) else "DIFF", flush=True)
    bad = np.nonzero(act != exd)[0]
    if len(bad):
        print("mismatch by expected action",
              {int(k): int(v) for k, v in zip(*np.unique(ex[bad], return_counts=True))},
              "first", bad[:8], act[bad[:8]], ex[bad[:8]], flush=True)


if __name__ == "__main__":
    main()
