#!/usr/bin/env python3
# SPDX-License-Identifier: GPL-2.0
"""Headline benchmark: device-resident parse + checksum + jhash + verdict on
BASELINE.json config 2 (16 M synthetic 64 B IPv4/UDP frames in one packed
UMEM pool, xdpsock geometry), one pool shard per GPU (config 5 at N > 1).

    python bench.py [--gpus N] [--steps K] [--warmup W]

--gpus N > 1 with no rank environment: this process only launches N child
ranks (one per GPU, rendezvous on 127.0.0.1) and returns the first failure's
code; under torch.distributed.run (WORLD_SIZE set) it is one of the ranks.

A step = one RX launch (xdp_rx_db_kernel: one block per CU, the tile loop
and the deferred-frame tail in one kernel) over the whole 16 M-frame shard
resident in HBM.  Timing: W untimed steps, barrier + synchronize, K timed
steps, synchronize + barrier, max over ranks.  value = frames processed by
all ranks / that time (Mpps, whole job).  The roofline figure is the
algorithmic bytes of a launch (113 B/frame) over the
launch's kernel time from HIP events recorded on the launch stream around
the kernel (xdpgpu_kernel_times), in a second pass of K launches on a
context with XDPGPU_CFG_TIMING so the events do not perturb the timed
steps.  traffic is the HBM bytes per launch from the committed rocprofv3
PMC summary (profiles/r<NN>_pmc.json, tools/pmc_profile.sh).  The CPU baseline
(rank 0 at N = 1 only, on a bounded sample, one pinned thread then one
thread per CPU the job may use) is the same per-frame work with the
reference headers' own checksum and jhash routines (oracle/_ref, compiled
from /root/reference in the container; kind "reference"), when that
library is present; the lean port (oracle/cpu_leg.c: the same outputs as
the oracle, checked on the sample) is timed beside it as port_mpps, with
the CPU model and the calibration probe.  Secondary lines: config 2 geometry
at 1500 B, config 3 (16 M IMIX, 44 B network_tuple), config 4 (16 M x
128 B nat64 ingress, static and dynamic state), multi-buffer 9000 B
packets, the ICMPv6 echo responder and the SYN proxy (8 M SYNs answered
with SYN-ACKs).
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "bpf-examples_amd"))

import torch  # noqa: E402  (before libxdpgpu: one HIP runtime)
import torch.distributed as dist  # noqa: E402

import shard  # noqa: E402
import xdpgpu  # noqa: E402

BYTES_PER_FRAME = 16 + 64 + 16 + 16 + 1   # desc + frame + result + tuple + verdict
RX_KERNELS = ("xdp_rx_db_kernel",)
HBM_PEAK_GBS = 8000.0                      # MI355X HBM3E, MI355X_MICROARCH.md
# the rendezvous and every control collective of the N-rank path end with
# an error after this long instead of hanging (XDPGPU_BENCH_PG_TIMEOUT)
PG_TIMEOUT_S = int(os.environ.get("XDPGPU_BENCH_PG_TIMEOUT", "600"))
METRIC = ("Mpps + GB/s device-resident parse+csum+jhash, 64B & 1500B frames, "
          "1/2/4/8 GPU")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def to_dev(a: np.ndarray, dev, pad: int = 64) -> torch.Tensor:
    t = torch.empty(a.nbytes + pad, dtype=torch.uint8, device=dev)
    t[a.nbytes:].zero_()
    t[: a.nbytes].copy_(torch.from_numpy(a.view(np.uint8).reshape(-1)))
    return t


_SETTLE = {}


def settle(dev, stream):
    """After a leg's device-to-device restore of its pool (outside the timed
    region): read 1 GiB of another buffer and synchronize, so that the
    restore's last writes, still dirty in the caches (the 256 MB Infinity
    Cache holds a quarter of a restored 1 GiB pool), are written back
    before the timed launch; otherwise their write-back lands in the
    launch (the echo leg: 0.352 vs 0.378 ms, tools/restore_probe.py).  The
    inputs are then resident in HBM, as the metric takes them."""
    buf = _SETTLE.get(dev)
    if buf is None:
        buf = _SETTLE[dev] = torch.ones(128 << 20, dtype=torch.int64, device=dev)
    with torch.cuda.stream(stream):
        buf[:1].copy_(buf.sum().view(1))
    torch.cuda.synchronize()


def out_sets(n: int, tuple_bytes: int, dev, sets: int = 2) -> list:
    """One (verdict, record, tuple) output set per slot in flight."""
    return [(torch.empty(n, dtype=torch.uint8, device=dev),
             torch.empty(n * 16, dtype=torch.uint8, device=dev),
             torch.empty(n * tuple_bytes, dtype=torch.uint8, device=dev))
            for _ in range(sets)]


def time_device(ctx, d_umem, usize, d_desc, n, outs, steps, warmup, world, in_flight=2):
    """W untimed + K timed launches between barrier + synchronize, as a
    device-resident RX loop keeps `in_flight` batches in flight: with 2,
    launch k goes to slot k mod 2 (xdpgpu_submit_dev: that slot's stream
    and scratch) with that slot's output set, so that a launch starts on
    the CUs the one before leaves while its last tiles finish (config 2:
    2-4 % a step; 16 M x 1500 B and IMIX, whose launches are 15x and 6x
    longer, run slower so and keep one in flight).  Returns
    (wall seconds, GPU span of the K timed launches in ms): one event on
    slot 0's stream before the first launch (slot 1's stream waits for it)
    and one on each slot's stream after the last, none between launches."""
    dev = d_umem.device
    ss = [torch.cuda.ExternalStream(ctx.slot_stream(i), device=dev) for i in range(2)]

    def launch(k):
        slot = k % in_flight
        v, r, t = outs[slot]
        ctx.submit_dev(slot, d_umem, usize, d_desc, n, v, r, t)

    torch.cuda.synchronize()   # the inputs, made on torch's streams
    for k in range(warmup):
        launch(k)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = [torch.cuda.Event(enable_timing=True) for _ in ss]
    e0.record(ss[0])
    ss[1].wait_event(e0)
    t0 = time.perf_counter()
    for k in range(steps):
        launch(k)
    for e, st in zip(e1, ss):
        e.record(st)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    span = max(e0.elapsed_time(e) for e in e1)
    if world > 1:
        dist.barrier()
    return t1 - t0, span


def outputs_ok(outs, expect) -> bool:
    """Every output set's verdicts equal the generator's (each set was
    written by timed launches)."""
    return all(bool(np.array_equal(v.cpu().numpy(), expect)) for v, _, _ in outs)


def kernel_breakdown(tctx, d_umem, usize, d_desc, n, d_v, d_res, d_tup, stream,
                     steps):
    """Per-kernel average ms from the HIP events the library records on the
    launch stream around each kernel (a context with CFG_TIMING; one launch
    at a time on one stream, a pass of its own before the timed steps, so
    the events do not perturb them: the kernel's own duration, which
    rocprofv3 reports for these launches)."""
    tctx.process_dev(d_umem, usize, d_desc, n, d_v, d_res, d_tup, stream)
    torch.cuda.synchronize()
    tctx.kernel_times()
    for _ in range(steps):
        tctx.process_dev(d_umem, usize, d_desc, n, d_v, d_res, d_tup, stream)
    torch.cuda.synchronize()
    return tctx.kernel_times()


def device_identity(local: int) -> dict:
    """What this rank runs on: the device's PCI bus id and UUID (the
    distinct-device check), its name, and the RCCL version torch carries
    (the "nccl" backend is RCCL on ROCm)."""
    p = torch.cuda.get_device_properties(local)
    try:
        rccl = ".".join(str(x) for x in torch.cuda.nccl.version())
    except Exception as e:  # noqa: BLE001 (reported, not fatal: gloo runs)
        rccl = f"unavailable ({type(e).__name__})"
    return {"local_rank": local, "name": p.name,
            "pci_bus_id": f"{getattr(p, 'pci_domain_id', 0):04x}:{p.pci_bus_id:02x}:"
                          f"{getattr(p, 'pci_device_id', 0):02x}",
            "uuid": str(getattr(p, "uuid", "")), "rccl": rccl}


def check_distinct_devices(idents: list, rehearse: bool) -> None:
    """One rank per GPU: two ranks on one device would time each other's
    launches as their own (the scaling curve would be wrong, not slow), so
    unless rehearsing that is an error naming the ranks.  Two ranks share a
    device when both their UUIDs and their PCI bus ids match, so that a
    driver reporting one UUID (or one bus id) for every device does not stop
    a run on distinct GPUs."""
    if rehearse:
        return
    seen = {}
    for r, d in enumerate(idents):
        key = (d.get("uuid") or "", d["pci_bus_id"])
        if key in seen:
            raise SystemExit(f"ranks {seen[key]} and {r} share device {d['pci_bus_id']} "
                             f"({key}): one rank per GPU (XDPGPU_BENCH_REHEARSE=1 rehearses "
                             "ranks sharing GPUs)")
        seen[key] = r


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(umem, descs, flags, fmt, budget_s: float = 10.0):
    """The CPU baseline on this host's cores: the reference headers'
    routines (oracle/_ref ref_leg_bench, kind "reference") when present,
    beside the lean port (oracle/cpu_leg.c, port_mpps); one pinned thread,
    then one thread per CPU the job may use; outputs checked against the
    oracle on part of the sample; the calibration probe (the survey probe's
    work) on both."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    oracle.lib()
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    # the cgroup's CPU quota, when it is below the affinity set (a GPU box's
    # share of its host): more threads than that only time-slice
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    cores = min(affinity, quota) if quota else affinity
    sample = descs[: 1 << 21]
    one = sample[: 1 << 19]
    t1, _ = oracle.leg_bench(umem, one, 1, 1, True, flags, 0, fmt)
    reps1 = max(1, int(3.0 / max(t1, 1e-3)))
    t1, _ = oracle.leg_bench(umem, one, 1, reps1, True, flags, 0, fmt)
    st_mpps = len(one) * reps1 / t1 / 1e6
    dt, _ = oracle.leg_bench(umem, sample, cores, 2, True, flags, 0, fmt)
    reps = max(1, int(2 * budget_s / max(dt, 1e-3)))
    dt, (v, res, tup) = oracle.leg_bench(umem, sample, cores, reps, True, flags, 0, fmt)
    mpps = len(sample) * reps / dt / 1e6
    k = 1 << 16
    ov, ores, otup, _ = oracle.process(umem, sample[:k], flags, 0, fmt)
    checked = bool(np.array_equal(v[:k], ov) and
                   res[:k].tobytes() == ores.tobytes() and
                   tup[: k * xdpgpu.TUPLE_BYTES[fmt]].tobytes() == otup.tobytes())
    mine, ref = oracle.probe_pair(umem, sample[: 1 << 20], 3)
    cal = {"probe": "parse + IPv4 csum + UDP csum + jhash(13 B), 1 thread",
           "leg_mpps": round((1 << 20) / mine / 1e6, 1),
           "reference_headers_mpps": round((1 << 20) / ref / 1e6, 1) if ref else None}
    if ref:
        cal["leg_over_reference"] = round(ref / mine, 3)
    # the same work with the reference headers' own routines (checksums
    # verified and recomputed as two passes each, as the reference idiom
    # does; oracle/ref_harness.c ref_leg_bench), on the same threads
    refleg = None
    r1 = oracle.ref_leg_bench(umem, one, 1, 1, True, flags, 0, fmt)
    if r1 is not None:
        rr1 = max(1, int(3.0 / max(r1[0], 1e-3)))
        r1 = oracle.ref_leg_bench(umem, one, 1, rr1, True, flags, 0, fmt)
        rdt, _ = oracle.ref_leg_bench(umem, sample, cores, 2, True, flags, 0, fmt)
        rreps = max(1, int(budget_s / max(rdt, 1e-3)))
        rdt, (rv, rres, rtup) = oracle.ref_leg_bench(umem, sample, cores, rreps, True, flags,
                                                     0, fmt)
        rmpps = len(sample) * rreps / rdt / 1e6
        refleg = {"reference_mpps": round(rmpps, 2),
                  "reference_single_thread_mpps": round(len(one) * rr1 / r1[0] / 1e6, 2),
                  "reference_outputs_match_leg": bool(
                      np.array_equal(rv, v) and rres.tobytes() == res.tobytes()),
                  "leg_over_reference": round(mpps / rmpps, 3),
                  "reference_sample": f"{len(sample)} frames x {rreps} passes on {cores} "
                                      f"threads ({rdt:.1f} s): lib_checksum.h ip_fast_csum / "
                                      "udp_csum and jhash.h jhash compiled from the reference "
                                      "(oracle/_ref), parse restated"}
    legs = cpu_legs(oracle)
    out = {"value": round(mpps, 2), "unit": "Mpps", "cores": cores,
            "affinity_cpus": affinity, "cgroup_cpu_quota": quota,
            "kind": "port", "cpu_model": cpu_model(),
            "gbps": round(mpps * 1e6 * BYTES_PER_FRAME / 1e9, 2),
            "single_thread_mpps": round(st_mpps, 2),
            "outputs_match_oracle": checked, "calibration": cal,
            "secondary_legs_1thread": legs,
            "sample": f"{len(sample)} config-2 frames x {reps} passes of oracle/cpu_leg.c "
                      f"(gcc -O2) on {cores} threads pinned one per CPU ({dt:.1f} s); "
                      f"1 pinned thread: {len(one)} frames x {reps1} passes"}
    if refleg:
        out.update(refleg)
        # the reference's own routines are the CPU path north_star names:
        # they are the baseline; the port (one pass per checksum, 64-bit
        # sums) stays beside them as port_mpps
        out["port_mpps"] = out["value"]
        out["port_sample"] = out["sample"]
        out["value"] = refleg["reference_mpps"]
        out["kind"] = "reference"
        out["gbps"] = round(refleg["reference_mpps"] * 1e6 * BYTES_PER_FRAME / 1e9, 2)
        out["single_thread_mpps"] = refleg["reference_single_thread_mpps"]
        out["sample"] = refleg["reference_sample"]
    return out


def cpu_legs(oracle) -> dict:
    """Single-thread CPU rates beside the secondary GPU lines, on samples
    of the same generators: IMIX through the lean leg (its fast shape, the
    oracle for the rest) and the SYN proxy through its oracle restatement
    (a loop-for-loop port of xdp_synproxy_kern.c).  nat64 has none: its
    oracle searches the state table linearly (a test checker, not a CPU
    form of the translator)."""
    out = {}
    u, d, _ = xdpgpu.pool_generate(1 << 18, xdpgpu.POOL_IMIX, 64, 0x5EED0003)
    t, _ = oracle.leg_bench(u, d, 1, 3, True, xdpgpu.CFG_DEFAULT, 0, xdpgpu.TUPLE_NET)
    out["imix_leg_mpps"] = round(3 * len(d) / t / 1e6, 2)
    u, d = synflood_pool(1 << 18, 0x5EED0007)
    c = xdpgpu.SynproxyCfg()
    c.ports[0] = 80
    c.now_ns = 10**18
    c.tailroom = 128 - 74
    t0 = time.perf_counter()
    oracle.synproxy(u, d, c)
    out["synproxy_oracle_mpps"] = round(len(d) / (time.perf_counter() - t0) / 1e6, 2)
    out["threads"] = 1
    return out


def pmc_traffic(n: int, size: int):
    """(HBM bytes per RX launch, source file) from the newest committed
    rocprofv3 PMC summary of config 2 (profiles/r<NN>_pmc.json,
    tools/pmc_profile.sh + tools/pmc_summary.py) when it was taken on this
    workload, else (None, None).  It was measured on the committed kernel
    of that round, not in this run."""
    import glob
    # the config-2 summaries only (r<NN>_pmc.json; the other workloads'
    # are r<NN>_pmc_<workload>.json)
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_pmc.json")))
    if not files:
        return None, None
    try:
        with open(files[-1]) as f:
            d = json.load(f)
        if d.get("frames") != n or d.get("frame_size") != size:
            return None, None
        return d.get("hbm_bytes_per_launch"), "profiles/" + os.path.basename(files[-1])
    except Exception:
        return None, None


def pmc_leg_traffic(pattern: str, frames: int):
    """HBM bytes per launch of a secondary leg from the newest committed PMC
    summary matching pattern (profiles/r<NN>_pmc_<workload>.json), scaled
    to the leg's frame count when the summary was taken on fewer frames of
    the same pool (the 1500 B leg lays its 2 M-frame pool down 8x): a dict
    with the bytes, the ratio to the leg's algorithmic bytes is the
    caller's; None when no summary exists."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)))
    if not files:
        return None
    try:
        with open(files[-1]) as f:
            d = json.load(f)
        b = float(d["hbm_bytes_per_launch"])
        pf = int(d.get("frames") or frames)
        return {"hbm_bytes_per_launch": b * frames / pf, "source": os.path.basename(files[-1]),
                "pmc_frames": pf}
    except Exception:
        return None


def attach_traffic(leg: dict, pattern: str, frames: int) -> dict:
    t = pmc_leg_traffic(pattern, frames)
    if t and leg.get("algorithmic_bytes_per_launch"):
        t["over_algorithmic"] = round(t["hbm_bytes_per_launch"] /
                                      leg["algorithmic_bytes_per_launch"], 3)
        t["hbm_bytes_per_launch"] = int(t["hbm_bytes_per_launch"])
    if t:
        # measured by rocprofv3 --pmc on the committed kernel of the
        # profile's round, not in this run (hence its own key)
        t["source"] = "profiles/" + t["source"]
        leg["committed_pmc_traffic"] = t
    return leg


def kt_round(kt: dict) -> dict:
    """The launch's HIP-event time: one RX launch is one kernel
    (xdp_rx_db_kernel), and the library records one event before it and
    one after it on the launch stream.  `launch_ms` is what
    `roofline.achieved` divides by; the rocprofv3 --kernel-trace --stats
    summary of the same command (profiles/r<NN>_kernel_stats_bench.csv)
    gives the kernel's average duration to compare.  (Until round 4 the
    library recorded two further empty pairs after the kernel, and the span
    to the last of them read ~3 % above the kernel.)"""
    return {"launches": kt["launches"], "launch_ms": round(kt["total_ms"], 4),
            "kernel_event_ms": round(kt["fast_ms"], 4)}


def side_run(ctx, tctx, dev, stream, n, kind, size, seed, fmt, steps, label, bpf_fn,
             replicate=1, world=1, rank=0, in_flight=1):
    """One secondary workload: pool, kernel event pass, K timed launches
    (`in_flight` slots, barrier-bracketed over the ranks when world > 1),
    verdict check.  replicate > 1: a pool of n frames is generated on the
    host and laid down `replicate` times back to back in HBM (descriptors
    offset by the copy's base), so that a multi-GB pool costs one host
    generation and copy; n * replicate frames are processed per launch.
    With world > 1 every rank runs its own shard (the caller offsets the
    seed by rank) and the rate is all ranks' frames over the slowest rank's
    time, as for config 2; `per_rank` lists each rank's numbers."""
    u, ds, ex = xdpgpu.pool_generate(n, kind, size, seed)
    if replicate > 1:
        g_umem = torch.empty(u.nbytes * replicate + 64, dtype=torch.uint8, device=dev)
        g_umem[u.nbytes * replicate:].zero_()
        src = torch.from_numpy(u).to(dev)
        g_umem[: u.nbytes * replicate].view(replicate, u.nbytes).copy_(
            src.unsqueeze(0).expand(replicate, -1))
        del src
        rd = np.tile(ds, replicate)
        rd["addr"] += np.repeat(np.arange(replicate, dtype=np.uint64) * np.uint64(u.nbytes),
                                len(ds))
        ds, ex, n = rd, np.tile(ex, replicate), n * replicate
    else:
        g_umem = to_dev(u, dev)
    del u
    g_desc = to_dev(ds, dev, 0)
    outs = out_sets(n, xdpgpu.TUPLE_BYTES[fmt], dev, in_flight)
    usize = g_umem.numel() - 64
    kt = kernel_breakdown(tctx, g_umem, usize, g_desc, n, *outs[0], None, steps)
    w, span = time_device(ctx, g_umem, usize, g_desc, n, outs, steps, 2, world, in_flight)
    ok = outputs_ok(outs, ex)
    algo = bpf_fn(ds)
    mine = {"rank": rank, "in_flight": in_flight, "ms_per_launch": round(w / steps * 1e3, 4),
            "gpu_span_ms_per_launch": round(span / steps, 4),
            "mpps": round(n * steps / w / 1e6, 1), "verdicts_ok": ok}
    per_rank = gather_ranks(mine, world)
    w_max = max(r["ms_per_launch"] for r in per_rank) * steps * 1e-3
    span_max = max(r["gpu_span_ms_per_launch"] for r in per_rank)
    out = {"workload": label, "frames": n, "n_gpus": world,
           "mpps": round(n * world * steps / w_max / 1e6, 1),
           "algorithmic_bytes_per_launch": int(algo),
           "ms_per_launch": round(w_max / steps * 1e3, 4),
           "gbps": round(algo * world / w_max * steps / 1e9, 1),
           "roofline_frac": round(algo / w_max * steps / 1e9 / HBM_PEAK_GBS, 4),
           # the same bytes over the timed launches' GPU span (events at
           # the ends of the K launches only)
           "roofline_frac_span": round(algo / (span_max * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           # and over the kernel's own duration (its event pair, one launch
           # at a time: kernel_times() averages over its launches)
           "roofline_frac_kernel": round(algo / (kt["total_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "kernel_ms": kt_round(kt),
           "verdicts_ok": all(r["verdicts_ok"] for r in per_rank)}
    if world > 1:
        out["per_rank"] = per_rank
    del g_umem, g_desc, outs
    torch.cuda.empty_cache()
    return out


def gather_ranks(mine: dict, world: int) -> list:
    """Every rank's small result dict, in rank order (all_gather_object;
    the rank's own alone at world 1)."""
    if world <= 1:
        return [mine]
    got = [None] * world
    dist.all_gather_object(got, mine)
    return got


def nat64_run(dev, stream, n, steps, local):
    """Config 4: nat64 ingress (IPv6 -> IPv4) over n 128 B frames.  The
    transform rewrites the UMEM, so every step restores the pool from a
    pristine device copy first (device-to-device, outside the timed
    region); each launch is timed with HIP events on its stream."""
    cfg, smap = xdpgpu.nat64_pool_config(xdpgpu.NAT64_INGRESS)
    u, ds, ex = xdpgpu.pool_generate(n, xdpgpu.POOL_NAT64, 128, 0x5EED0004)
    pristine = to_dev(u, dev)
    work = torch.empty_like(pristine)
    d_desc = to_dev(ds, dev, 0)
    d_act = torch.empty(n, dtype=torch.uint8, device=dev)
    d_out = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    ms = []
    with xdpgpu.XdpGpu(local) as g:
        g.nat64_setup(cfg, smap)
        for k in range(steps + 2):
            with torch.cuda.stream(stream):
                work.copy_(pristine, non_blocking=True)
            settle(dev, stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            g.nat64_dev(work, u.nbytes, d_desc, n, d_act, d_out, stream)
            e1.record(stream)
            torch.cuda.synchronize()
            if k >= 2:
                ms.append(e0.elapsed_time(e1))
    ok = bool(np.array_equal(d_act.cpu().numpy(), ex))
    # dynamic state (alloc_new_state) in steady state: the 65533 static
    # mappings, the v4 pool widened to 10.98.0.0/15 so that the pool's 1000
    # unmapped sources get addresses from next_addr 1 (10.98.0.x) in the
    # untimed first launches; then every launch is a hit per frame (the
    # last_seen stamps, the listed-frame count read back)
    dms = []
    dcfg = xdpgpu.Nat64Cfg.from_buffer_copy(bytes(cfg))
    dcfg.v4_prefix, dcfg.v4_mask = 0x0A620000, 0xFFFE0000
    with xdpgpu.XdpGpu(local) as g:
        g.nat64_setup(dcfg, smap)
        g.nat64_dynamic(7200 * 10**9, 1)
        for k in range(steps + 2):
            g.nat64_clock(10**13 + k)
            with torch.cuda.stream(stream):
                work.copy_(pristine, non_blocking=True)
            settle(dev, stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            g.nat64_dev(work, u.nbytes, d_desc, n, d_act, d_out, stream)
            e1.record(stream)
            torch.cuda.synchronize()
            if k >= 2:
                dms.append(e0.elapsed_time(e1))
        nent = len(g.nat64_state()[0])
    exd = ex.copy()
    exd[exd == xdpgpu.NAT64_NO_STATE] = xdpgpu.TC_ACT_REDIRECT
    dyn = {"workload": "the same pool, dynamic state: 65533 static entries + those allocated for "
                       "its unmapped sources (v4 pool 10.98.0.0/15), steady state",
           "ms_per_launch": round(float(np.mean(dms)), 4),
           "entries": nent, "actions_ok": bool(np.array_equal(d_act.cpu().numpy(), exd))}
    t = float(np.mean(ms))
    algo = n * 149
    out = {"workload": f"config4: {n} x 128B IPv6 frames, nat64 ingress (64:ff9b::/96, "
                       "65533 static mappings)",
           "frames": n, "mpps": round(n / t / 1e3, 1), "kernel_ms": round(t, 4),
           "algorithmic_bytes_per_launch": algo,
           "gbps": round(algo / t / 1e6, 1),
           "roofline_frac": round(algo / t / 1e6 / HBM_PEAK_GBS, 4),
           "actions_ok": ok, "dynamic_state": dyn}
    del pristine, work, d_desc, d_act, d_out
    torch.cuda.empty_cache()
    return out


def synflood_pool(n: int, seed: int):
    """n IPv4 SYNs (74 B: MSS, SACK_PERM, timestamp, window scale options,
    a Linux client's SYN) at a 128-byte stride, random source address, port,
    sequence number and timestamp, valid checksums; SYN proxy leg."""
    rng = np.random.default_rng(seed)
    t = np.zeros((n, 74), np.uint8)
    t[:, 0:14] = np.frombuffer(bytes([2, 0, 0, 0, 0, 1, 2, 0, 0, 0, 0, 2, 8, 0]), np.uint8)
    t[:, 14:34] = np.frombuffer(bytes([0x45, 0, 0, 60, 0, 0, 0x40, 0, 64, 6, 0, 0,
                                       10, 0, 0, 0, 10, 1, 0, 1]), np.uint8)
    src = rng.integers(0, 1 << 16, n)
    t[:, 28], t[:, 29] = src >> 8, src & 0xFF
    t[:, 34:74] = np.frombuffer(bytes([0, 0, 0, 80, 0, 0, 0, 0, 0, 0, 0, 0, 0xA0, 0x02,
                                       0xFF, 0xFF, 0, 0, 0, 0, 2, 4, 5, 0xB4, 4, 2, 8, 10,
                                       0, 0, 0, 0, 0, 0, 0, 0, 1, 3, 3, 7]), np.uint8)
    sport = rng.integers(1024, 1 << 16, n)
    t[:, 34], t[:, 35] = sport >> 8, sport & 0xFF
    t[:, 38:42] = rng.integers(0, 256, (n, 4), dtype=np.uint8)      # seq
    t[:, 62:66] = rng.integers(0, 256, (n, 4), dtype=np.uint8)      # TSval

    def csum(words):
        s = words.sum(1, dtype=np.uint64)
        while True:
            hi = s >> np.uint64(16)
            if not hi.any():
                break
            s = (s & np.uint64(0xFFFF)) + hi
        return (~s.astype(np.uint32)) & 0xFFFF

    def be_words(a):
        a = a.astype(np.uint32)
        return (a[:, 0::2] << 8) | a[:, 1::2]

    c = csum(be_words(t[:, 14:34]))
    t[:, 24], t[:, 25] = c >> 8, c & 0xFF
    pseudo = np.concatenate([be_words(t[:, 26:34]),
                             np.full((n, 1), 6 + 40, np.uint32)], 1)
    c = csum(np.concatenate([be_words(t[:, 34:74]), pseudo], 1))
    t[:, 50], t[:, 51] = c >> 8, c & 0xFF
    umem = np.zeros(n * 128 + 64, np.uint8)
    umem[:n * 128].reshape(n, 128)[:, :74] = t
    descs = np.zeros(n, xdpgpu.DESC_DTYPE)
    descs["addr"] = np.arange(n, dtype=np.uint64) * 128
    descs["len"] = 74
    return umem, descs


def synproxy_run(dev, stream, n, steps, local):
    """SYN proxy (xdp_synproxy_kern.c): n SYNs answered in place with
    SYN-ACKs.  Like nat64, the pool is restored from a pristine device
    copy before each launch (outside the timed region)."""
    u, ds = synflood_pool(n, 0x5EED0007)
    pristine = to_dev(u, dev)
    work = torch.empty_like(pristine)
    d_desc = to_dev(ds, dev, 0)
    d_v = torch.empty(n, dtype=torch.uint8, device=dev)
    d_out = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    d_cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    c = xdpgpu.SynproxyCfg()
    c.ports[0] = 80
    c.now_ns = 10**18
    c.tailroom = 128 - 74
    c.cookie_key = 0x5EED
    ms = []
    with xdpgpu.XdpGpu(local) as g:
        for k in range(steps + 2):
            with torch.cuda.stream(stream):
                work.copy_(pristine, non_blocking=True)
            settle(dev, stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            g.synproxy_dev(work, u.nbytes, d_desc, n, c, d_v, d_out, d_cnt, stream)
            e1.record(stream)
            torch.cuda.synchronize()
            if k >= 2:
                ms.append(e0.elapsed_time(e1))
    v = d_v.cpu().numpy()
    t = float(np.mean(ms))
    # read 16 (descriptor) + 74 (SYN), write 74 (SYN-ACK) + 16 (descriptor) + 1
    algo = n * (16 + 74 + 74 + 16 + 1)
    out = {"workload": f"{n} x 74B IPv4 SYNs (MSS/SACK/TS/WS options) at a 128B stride, "
                       "SYN-ACK written in place (xdp_synproxy_kern.c)",
           "frames": n, "mpps": round(n / t / 1e3, 1), "kernel_ms": round(t, 4),
           "algorithmic_bytes_per_launch": algo, "gbps": round(algo / t / 1e6, 1),
           "roofline_frac": round(algo / t / 1e6 / HBM_PEAK_GBS, 4),
           "all_synack": bool((v == 3).all())}
    del pristine, work, d_desc, d_v, d_out
    torch.cuda.empty_cache()
    return out


def frags_run(dev, stream, n, steps, local, size=9000, chunk=4096):
    """Multi-buffer packets (XDPGPU_CFG_FRAGS): n jumbo frames, each cut in
    place into fragments of at most `chunk` bytes (XDP_PKT_CONTD on all but
    the last).  Times the whole launch (count, RX kernels over the gathered
    packets, scatter) and checks every fragment's verdict against the
    generator's verdict for its frame."""
    u, d, ex = xdpgpu.pool_generate(n, xdpgpu.POOL_UDP4, size, 0x5EED0022)
    lens = d["len"].astype(np.int64)
    nf = (lens + chunk - 1) // chunk
    frame_of = np.repeat(np.arange(n), nf)
    k = np.arange(len(frame_of)) - np.repeat(np.cumsum(nf) - nf, nf)
    fd = np.zeros(len(frame_of), xdpgpu.DESC_DTYPE)
    fd["addr"] = d["addr"][frame_of] + k * chunk
    fd["len"] = np.minimum(lens[frame_of] - k * chunk, chunk)
    fd["options"] = np.where(k < nf[frame_of] - 1, xdpgpu.PKT_CONTD, 0)
    m = len(fd)
    g_umem = to_dev(u, dev)
    g_desc = to_dev(fd, dev, 0)
    outs = out_sets(m, 16, dev, 1)
    with xdpgpu.XdpGpu(local, xdpgpu.CFG_DEFAULT | xdpgpu.CFG_FRAGS, 0, xdpgpu.TUPLE_V4,
                       64) as g:
        w, _ = time_device(g, g_umem, u.nbytes, g_desc, m, outs, steps, 2, 1, 1)
    ok = outputs_ok(outs, ex[frame_of])
    t = w / steps
    out = {"workload": f"{n} x {size}B IPv4/UDP packets in {chunk}B fragments "
                       f"({m} descriptors), XDPGPU_CFG_FRAGS",
           "packets": n, "descriptors": m, "mpps": round(n / t / 1e6, 1),
           "ms_per_launch": round(t * 1e3, 4),
           "packet_gbps": round(float(lens.sum()) / t / 1e9, 1), "verdicts_ok": ok}
    # descriptors in, packet bytes, verdict + record + tuple out per descriptor
    algo = m * (16 + 1 + 16 + 16) + int(lens.sum())
    out.update({"algorithmic_bytes_per_launch": algo, "gbps": round(algo / t / 1e9, 1),
                "roofline_frac": round(algo / t / 1e9 / HBM_PEAK_GBS, 4)})
    del g_umem, g_desc, outs
    torch.cuda.empty_cache()
    return out


def echo_run(dev, stream, n, steps, local, size=128, ppm=200000, tune=0, window=0):
    """The ICMPv6 echo responder (af_xdp_user.c:968-1040) as a throughput
    mode: n frames of which ppm / 1e6 are echo requests, rewritten in place
    into replies (TX).  The rewrite changes the UMEM, so every step
    restores the pool from a pristine device copy first (outside the timed
    region); each launch is timed with HIP events on its stream."""
    u, ds, ex = xdpgpu.pool_generate(n, xdpgpu.POOL_UDP4, size, 0x5EED0042,
                                     ppm_echo6=ppm)
    # the generator expects REDIRECT for a request (no responder): TX here
    eff = (ds["addr"] & ((1 << 48) - 1)) + (ds["addr"] >> 48)
    req = ((u[eff + 12] == 0x86) & (u[eff + 13] == 0xDD) & (u[eff + 20] == 58) &
           (u[eff + 54] == 128) & (ds["len"] >= 62) & (ex == xdpgpu.REDIRECT))
    want = np.where(req, xdpgpu.TX, ex).astype(np.uint8)
    pristine = to_dev(u, dev)
    work = torch.empty_like(pristine)
    d_desc = to_dev(ds, dev, 0)
    d_v = torch.empty(n, dtype=torch.uint8, device=dev)
    d_res = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    d_tup = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    ms = []
    with xdpgpu.XdpGpu(local, xdpgpu.CFG_DEFAULT | xdpgpu.CFG_ICMP6_ECHO, 0,
                       xdpgpu.TUPLE_V4, window, tune=tune) as g:
        for k in range(steps + 2):
            with torch.cuda.stream(stream):
                work.copy_(pristine, non_blocking=True)
            settle(dev, stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            g.process_dev(work, u.nbytes, d_desc, n, d_v, d_res, d_tup, stream)
            e1.record(stream)
            torch.cuda.synchronize()
            if k >= 2:
                ms.append(e0.elapsed_time(e1))
    v = d_v.cpu().numpy()
    ok = bool(np.array_equal(v, want))
    t = float(np.mean(ms))
    ntx = int(req.sum())
    algo = n * (16 + 16 + 16 + 1) + int(ds["len"].astype(np.int64).sum()) + ntx * 64
    out = {"workload": f"{n} x {size}B frames, {ppm / 1e4:.0f} % ICMPv6 echo requests "
                       "answered in place (XDPGPU_CFG_ICMP6_ECHO)",
           "frames": n, "tx_frames": ntx, "mpps": round(n / t / 1e3, 1),
           "kernel_ms": round(t, 4), "algorithmic_bytes_per_launch": algo,
           "gbps": round(algo / t / 1e6, 1),
           "roofline_frac": round(algo / t / 1e6 / HBM_PEAK_GBS, 4), "verdicts_ok": ok}
    del pristine, work, d_desc, d_v, d_res, d_tup
    torch.cuda.empty_cache()
    return out


def pcie_ceiling(dev, mib: int = 256, reps: int = 10) -> dict:
    """What this box's PCIe link moves between page-locked host memory and
    HBM with plain copies (the ceiling the host path is priced against):
    H2D alone, D2H alone, and both at once on two streams, GB/s."""
    nb = mib << 20
    h_in = torch.empty(nb, dtype=torch.uint8, pin_memory=True)
    h_out = torch.empty(nb, dtype=torch.uint8, pin_memory=True)
    d_a = torch.empty(nb, dtype=torch.uint8, device=dev)
    d_b = torch.empty(nb, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps

    def h2d():
        with torch.cuda.stream(s1):
            d_a.copy_(h_in, non_blocking=True)

    def d2h():
        with torch.cuda.stream(s2):
            h_out.copy_(d_b, non_blocking=True)

    def both():
        h2d()
        d2h()

    t_in, t_out, t_both = timed(h2d), timed(d2h), timed(both)
    out = {"h2d_gbps": round(nb / t_in / 1e9, 1), "d2h_gbps": round(nb / t_out / 1e9, 1),
           "duplex_gbps": round(2 * nb / t_both / 1e9, 1),
           "probe": f"{mib} MiB page-locked copies, {reps} each, torch streams"}
    del h_in, h_out, d_a, d_b
    return out


def e2e_run(local, umem, descs, expect, B: int, nbatches: int, chunk: int, window: int,
            ceil: dict, flags: int = xdpgpu.CFG_DEFAULT, slots: int = 2) -> dict:
    """The host path as an RX loop drives it (xdpgpu_submit / xdpgpu_wait,
    two batches in flight): each batch's frames copied from the pinned host
    UMEM into the slot's device mirror (rows of chunks when chunk is given:
    xdpgpu_register_umem), its descriptors in, the kernel, verdicts,
    records and tuples back into page-locked per-slot buffers.  Batches of B
    consecutive descriptors cycle over the pool.  One pass checks every
    batch's verdicts, a second is timed; the PCIe bytes per frame come from
    xdpgpu_host_stats over the timed pass.  flags: XDPGPU_CFG_UMEM_GATHER
    moves a chunked UMEM's frames by the gather kernel instead; slots:
    batches in flight (xdpgpu_submit's slots, 2 = double buffering)."""
    n = len(descs)
    per = max(1, n // B)
    h = xdpgpu.XdpGpu(local, flags, 0, xdpgpu.TUPLE_V4, window, max_batch=B)
    h.register_umem(umem, chunk)
    threads = h.host_threads(0) if flags & xdpgpu.CFG_HOST_COMPACT else None
    # the descriptors as the RX ring holds them (page-locked), and
    # page-locked per-slot outputs, as an RX loop keeps them
    hd = xdpgpu.HostBuffer(per * B, xdpgpu.DESC_DTYPE)
    hd.array[:] = descs[: per * B]
    outs = [[xdpgpu.HostBuffer(B, dt) for dt in (np.uint8, xdpgpu.RESULT_DTYPE,
                                                 xdpgpu.TUPLE4_DTYPE)] for _ in range(slots)]

    def one_pass(check: bool):
        ok = True
        pending = [None] * slots
        t0 = time.perf_counter()
        for k in range(nbatches + slots):
            slot = k % slots
            if pending[slot] is not None:
                h.wait(slot)
                if check:
                    lo = pending[slot]
                    ok &= bool(np.array_equal(outs[slot][0].array, expect[lo:lo + B]))
                pending[slot] = None
            if k >= nbatches:
                continue
            lo = (k % per) * B
            v, r, t = (b.array for b in outs[slot])
            h.submit(slot, hd.array[lo:lo + B], v, r, t)
            pending[slot] = lo
        return time.perf_counter() - t0, ok

    _, ok = one_pass(True)
    s0 = h.host_stats()
    te, _ = one_pass(False)
    s1 = h.host_stats()
    h.close()
    hd.close()
    for o in outs:
        for b in o:
            b.close()
    fr = s1["frames"] - s0["frames"]
    h2d = (s1["umem_h2d_bytes"] - s0["umem_h2d_bytes"]) + (s1["desc_h2d_bytes"] -
                                                           s0["desc_h2d_bytes"])
    d2h = s1["out_d2h_bytes"] - s0["out_d2h_bytes"]
    h2d_gbps = h2d / te / 1e9
    d2h_gbps = d2h / te / 1e9
    return {"mpps": round(fr / te / 1e6, 1), "frames": fr, "batch": B, "batches": nbatches,
            "slots": slots, "chunk": chunk, "pinned_buffers": True,
            "umem_gather": bool(flags & xdpgpu.CFG_UMEM_GATHER) and
            s1["umem_gathers"] > s0["umem_gathers"],
            "host_compact": bool(flags & xdpgpu.CFG_HOST_COMPACT) and
            s1["umem_compacted"] > s0["umem_compacted"],
            **({"host_threads": threads,
                "pack_ms_per_batch": round((s1["compact_ns"] - s0["compact_ns"]) / 1e6 /
                                           max(1, s1["umem_compacted"] - s0["umem_compacted"]),
                                           3)} if threads else {}),
            "h2d_bytes_per_frame": round(h2d / fr, 1),
            "umem_copies_per_batch": round((s1["umem_copies"] - s0["umem_copies"]) /
                                           max(1, s1["batches"] - s0["batches"]), 1),
            "d2h_bytes_per_frame": round(d2h / fr, 1),
            "h2d_gbps": round(h2d_gbps, 1), "d2h_gbps": round(d2h_gbps, 1),
            "pcie_ceiling": ceil,
            "pcie_frac": round(max(h2d_gbps / ceil["h2d_gbps"], d2h_gbps / ceil["d2h_gbps"]), 3),
            "verdicts_ok": ok}


def huge_pages_copy(a: np.ndarray) -> np.ndarray:
    """a copied into anonymous memory advised for transparent huge pages
    (madvise MADV_HUGEPAGE): xdpsock maps its UMEM with MAP_HUGETLB in
    unaligned-chunk mode (AF_XDP-example/xdpsock.c:1246, :2062).  The
    array keeps the mapping alive."""
    import mmap
    mm = mmap.mmap(-1, max(a.nbytes, 1), flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    if hasattr(mm, "madvise") and hasattr(mmap, "MADV_HUGEPAGE"):
        mm.madvise(mmap.MADV_HUGEPAGE)
    out = np.frombuffer(mm, np.uint8)[: a.nbytes]
    out[:] = a.view(np.uint8).reshape(-1)
    return out


def thp_mode() -> str:
    try:
        with open("/sys/kernel/mm/transparent_hugepage/enabled") as f:
            return f.read().strip()
    except OSError:
        return "unknown"


def gather_leg(frames: int, batches: int, ceil: dict) -> dict:
    """e2e_run with XDPGPU_CFG_UMEM_GATHER on the chunked leg's workload,
    run by tools/e2e_probe.py as a child process (its own GPU context):
    the JSON of its gather line, or the failure."""
    cmd = [sys.executable, os.path.join(ROOT, "tools", "e2e_probe.py"), "--gather-only",
           "--no-submit-cost", "--frames", str(frames), "--batches", str(batches),
           "--h2d-ceil", str(ceil["h2d_gbps"]), "--d2h-ceil", str(ceil["d2h_gbps"])]
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    except subprocess.TimeoutExpired:
        return {"error": "timed out after 300 s"}
    for line in reversed(p.stdout.splitlines()):
        if line.startswith("{"):
            r = json.loads(line)
            r.pop("mode", None)
            r["pcie_ceiling"] = ceil
            r["process"] = "child (tools/e2e_probe.py)"
            return r
    return {"error": f"exit {p.returncode}: {p.stderr.strip()[-300:]}"}


def free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_envs(n: int, base: dict, port: int) -> list:
    """The environment of each of n ranks on this node, as
    torch.distributed.run sets it: one process per GPU (rank r drives
    cuda:r), rendezvous on 127.0.0.1."""
    envs = []
    for r in range(n):
        e = dict(base)
        e.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n),
                  "LOCAL_WORLD_SIZE": str(n), "GROUP_RANK": "0",
                  "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
        e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        envs.append(e)
    return envs


def launch_ranks(cmd: list, n: int, base_env: dict | None = None, poll_s: float = 0.2) -> int:
    """`bench.py --gpus N` without an outer launcher: start N fresh child
    processes of `cmd`, one per GPU (the reference's unit of scale is one
    XSK socket per RX queue, af_xdp_user.c:1542-1611; here one rank per
    GPU), and wait for them.  The parent is a pure launcher: it has touched
    neither the GPU nor libxdpgpu (nothing here initialises HIP), and it
    never execs itself.  If a rank fails, the others are terminated (a rank
    left waiting in a collective would never finish); the return code is
    the first failure's, else 0."""
    import signal
    envs = rank_envs(n, dict(os.environ if base_env is None else base_env), free_port())
    procs = [subprocess.Popen(cmd, env=e, start_new_session=True) for e in envs]
    rc = 0
    try:
        live = set(range(n))
        while live:
            for r in sorted(live):
                c = procs[r].poll()
                if c is None:
                    continue
                live.discard(r)
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 128 - c
                    log(f"[launcher] rank {r} exited with {c}: stopping the others")
                    for q in live:
                        try:
                            os.killpg(procs[q].pid, signal.SIGTERM)
                        except ProcessLookupError:
                            pass
            if live:
                time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                p.wait()
    return rc


def world_plan(gpus: int, env: dict, device_count: int, rehearse: bool) -> str:
    """What this process is for: "run" (a rank: the outer launcher's, ours,
    or N = 1) or "launch" (N > 1 and no rank environment: start N ranks).
    Raises when the world and --gpus disagree, or when fewer GPUs exist
    than ranks asked for (unless rehearsing: ranks then share GPUs)."""
    if gpus < 1:
        raise SystemExit(f"--gpus {gpus}: need at least 1")
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if world != gpus:
            raise SystemExit(f"WORLD_SIZE {world} but --gpus {gpus}: the launcher and the "
                             "bench disagree on the number of ranks")
        plan = "run"
    else:
        plan = "launch" if gpus > 1 else "run"
    if not rehearse and device_count < gpus:
        raise SystemExit(f"--gpus {gpus} but {device_count} GPU(s) visible: one rank per GPU "
                         "(set XDPGPU_BENCH_REHEARSE=1 to rehearse ranks sharing GPUs)")
    return plan


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--frames", type=int, default=16 << 20, help="frames per GPU")
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--window", type=int, default=0,
                    help="header window of every RX context: 64, 128, or 0 (the library "
                         "picks per batch: 128 when the UMEM holds >= 128 B a frame)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--legs", default="1500,imix,nat64,frags,echo,synproxy",
                    help="secondary workloads: comma list of 1500, imix, nat64, frags, echo")
    ap.add_argument("--frames-1500", type=int, default=2 << 20,
                    help="1500 B frames generated per GPU, laid down 8x in HBM")
    ap.add_argument("--imix-frames", type=int, default=16 << 20)
    ap.add_argument("--nat64-frames", type=int, default=16 << 20)
    ap.add_argument("--tune", type=lambda x: int(x, 0), default=0,
                    help="cfg.tune of the secondary legs' contexts (diagnostic A/B)")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip the end-to-end host path (pinned H2D + kernel + D2H)")
    ap.add_argument("--e2e-batches", type=int, default=32,
                    help="batches per timed pass of each host-path leg")
    ap.add_argument("--e2e-chunked-frames", type=int, default=1 << 20,
                    help="frames (4 KiB chunks) of the chunked host-path leg's UMEM; 0: skip")
    args = ap.parse_args()

    # XDPGPU_BENCH_REHEARSE=1: a rehearsal of the N-rank path on fewer GPUs
    # than ranks (ranks share devices, gloo for the control collectives);
    # its numbers are not a scaling measurement
    rehearse = os.environ.get("XDPGPU_BENCH_REHEARSE") == "1"
    # device_count() does not initialise the GPU on this image: the
    # launcher's children get a clean process each
    plan = world_plan(args.gpus, os.environ, torch.cuda.device_count(), rehearse)
    if plan == "launch":
        sys.exit(launch_ranks([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                              args.gpus))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if rehearse:
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)      # before RCCL binds the rank
    ident = device_identity(local)
    if world > 1:
        # an explicit timeout: a rank that never arrives (a dead device, a
        # rendezvous that cannot resolve) ends the job with an error
        # instead of a hang
        dist.init_process_group("gloo" if rehearse else "nccl",
                                timeout=datetime.timedelta(seconds=PG_TIMEOUT_S))
    dev = torch.device("cuda", local)
    idents = gather_ranks(ident, world)
    check_distinct_devices(idents, rehearse)
    log(f"[rank {rank}] {ident}")

    # config 2 shard (config 5 at N > 1: same per-GPU content, seed offset)
    t = time.time()
    n = args.frames
    umem, descs, expect = xdpgpu.pool_generate(n, xdpgpu.POOL_UDP4, args.size,
                                               shard.shard_seed(0x5EED0002, rank))
    log(f"[rank {rank}] pool {n} x {args.size} B generated in {time.time() - t:.1f} s")
    d_umem = to_dev(umem, dev)
    d_desc = to_dev(descs, dev, 0)
    outs = out_sets(n, 16, dev)
    ctx = xdpgpu.XdpGpu(local, xdpgpu.CFG_DEFAULT, 0, xdpgpu.TUPLE_V4, args.window)
    tctx = xdpgpu.XdpGpu(local, xdpgpu.CFG_DEFAULT | xdpgpu.CFG_TIMING, 0,
                         xdpgpu.TUPLE_V4, args.window)
    stream = torch.cuda.Stream(dev)

    # the kernel's own duration first (one launch at a time, an event pair
    # around each), then the W warmup and K timed steps
    kt = kernel_breakdown(tctx, d_umem, umem.nbytes, d_desc, n, *outs[0], None, args.steps)
    kms = kt["total_ms"]
    wall, span = time_device(ctx, d_umem, umem.nbytes, d_desc, n, outs, args.steps,
                             args.warmup, world)
    # correctness spot check of the timed outputs against the generator
    ok = outputs_ok(outs, expect)
    # max time / summed frames over ranks (no data-path collective)
    wall_max, total_frames, all_ok = shard.reduce_timing(wall, n * args.steps, ok,
                                                         None if rehearse else dev)
    per_rank = gather_ranks({"rank": rank, "device": ident["pci_bus_id"],
                             "ms_per_step": round(wall / args.steps * 1e3, 4),
                             "gpu_span_ms_per_step": round(span / args.steps, 4),
                             "kernel_ms": round(kms, 4),
                             "mpps": round(n * args.steps / wall / 1e6, 1),
                             "verdicts_ok": ok}, world)
    span_step = max(r["gpu_span_ms_per_step"] for r in per_rank)
    mpps = total_frames / wall_max / 1e6
    gbps = total_frames * BYTES_PER_FRAME / wall_max / 1e9
    # per GPU, over the timed launches: the slowest rank's GPU span a step
    achieved = BYTES_PER_FRAME * n / (span_step * 1e-3) / 1e9

    secondary = {}
    if not args.no_secondary:
        del d_umem, outs
        torch.cuda.empty_cache()
        steps2 = max(5, args.steps // 5)
        legs = set(args.legs.split(","))
        if "1500" in legs:
            # 1500 B frames (BASELINE metric names both sizes at 1/2/4/8
            # GPUs), config 2 geometry, 16 M frames per GPU as config 2
            # (25 GB: 2 M generated, laid down 8x); every rank its own
            # shard, seed offset by rank
            secondary["secondary_1500B"] = side_run(
                ctx, tctx, dev, stream, args.frames_1500, xdpgpu.POOL_UDP4, 1500,
                shard.shard_seed(0x5EED0012, rank), xdpgpu.TUPLE_V4, steps2,
                f"config2-geometry {8 * args.frames_1500} x 1500B IPv4/UDP per GPU (a "
                f"{args.frames_1500}-frame pool laid down 8x), V4 tuple",
                lambda ds: len(ds) * (16 + 16 + 16 + 1) + int(ds["len"].astype(np.int64).sum()),
                replicate=8, world=world, rank=rank)
            attach_traffic(secondary["secondary_1500B"], "r[0-9][0-9]_pmc_1500_w128.json",
                           8 * args.frames_1500)
        # the single-GPU configurations (BASELINE configs 3 and 4) and the
        # other modes: rank 0 at N = 1 only
        legs = legs if world == 1 else set()
        if "imix" in legs:
            # config 3: IMIX with the 44 B network_tuple (429.3 B/frame)
            ctx3 = xdpgpu.XdpGpu(local, xdpgpu.CFG_DEFAULT, 0, xdpgpu.TUPLE_NET, args.window)
            tctx3 = xdpgpu.XdpGpu(local, xdpgpu.CFG_DEFAULT | xdpgpu.CFG_TIMING, 0,
                                  xdpgpu.TUPLE_NET, args.window)
            secondary["config3_imix"] = side_run(
                ctx3, tctx3, dev, stream, args.imix_frames, xdpgpu.POOL_IMIX, 64, 0x5EED0003,
                xdpgpu.TUPLE_NET, steps2,
                f"config3: {args.imix_frames} IMIX frames (64/570/1500 7:4:1, VLAN, IPv6), "
                "network_tuple",
                lambda ds: len(ds) * (16 + 16 + 44 + 1) + int(ds["len"].astype(np.int64).sum()))
            attach_traffic(secondary["config3_imix"], "r[0-9][0-9]_pmc_config3_w128.json",
                           args.imix_frames)
            ctx3.close()
            tctx3.close()
        if "nat64" in legs:
            secondary["config4_nat64"] = nat64_run(dev, stream, args.nat64_frames, steps2,
                                                   local)
            attach_traffic(secondary["config4_nat64"], "r[0-9][0-9]_pmc_config4.json",
                           args.nat64_frames)
        if "frags" in legs:
            secondary["multibuffer_9000B"] = frags_run(dev, stream, 1 << 18, steps2, local)
        if "echo" in legs:
            secondary["icmp6_echo"] = echo_run(dev, stream, 8 << 20, steps2, local,
                                               tune=args.tune, window=args.window)
            attach_traffic(secondary["icmp6_echo"], "r[0-9][0-9]_pmc_echo_leg.json", 8 << 20)
        if "synproxy" in legs:
            secondary["synproxy"] = synproxy_run(dev, stream, 8 << 20, steps2, local)
            attach_traffic(secondary["synproxy"], "r[0-9][0-9]_pmc_synproxy_leg.json",
                           8 << 20)

    e2e = None
    e2e_chunked = None
    e2e_gather = None
    e2e_compact = None
    e2e_compact_huge = None
    if not args.no_e2e and rank == 0 and world == 1:
        ceil = pcie_ceiling(dev)
        # host path, the packed pool: pinned UMEM, H2D span + descs, kernel,
        # D2H outputs
        e2e = e2e_run(local, umem, descs, expect, 1 << 20, args.e2e_batches, 0,
                      args.window, ceil)
        e2e["workload"] = (f"config-2 frames from a packed 64B-stride host UMEM "
                           f"({umem.nbytes >> 20} MiB), batches cycling over it")
        if args.e2e_chunked_frames:
            # the reference's UMEM geometry: 4 KiB chunks (af_xdp_user.c:56-57,
            # xdpsock.c:133), each 64 B frame at its chunk's XDP_PACKET_HEADROOM
            nc = args.e2e_chunked_frames
            cu, cd, ce = xdpgpu.pool_generate(nc, xdpgpu.POOL_UDP4, args.size, 0x5EED0032,
                                              stride=4096, headroom=256)
            e2e_chunked = e2e_run(local, cu, cd, ce, nc // 2, args.e2e_batches, 4096,
                                  args.window, ceil)
            e2e_chunked["workload"] = (f"{nc} x {args.size}B IPv4/UDP frames in 4 KiB chunks "
                                       f"at headroom 256 ({cu.nbytes >> 20} MiB host UMEM, "
                                       "registered with chunk_size 4096), batches of half "
                                       "the UMEM cycling over it")
            # the same with XDPGPU_CFG_HOST_COMPACT: the host threads (the
            # CPUs the job may use, at most 16) pack each frame's bytes out
            # of its chunk into one page-locked buffer a batch, one transfer
            e2e_compact = e2e_run(local, cu, cd, ce, nc // 2, args.e2e_batches, 4096,
                                  args.window, ceil,
                                  flags=xdpgpu.CFG_DEFAULT | xdpgpu.CFG_HOST_COMPACT)
            e2e_compact["workload"] = e2e_chunked["workload"] + ", XDPGPU_CFG_HOST_COMPACT"
            # the same UMEM in transparent huge pages (xdpsock's MAP_HUGETLB
            # UMEM): one 4 KiB chunk a frame is one page walk a frame in 4 KiB
            # pages (tools/pack_probe.c)
            hu = huge_pages_copy(cu)
            e2e_compact_huge = e2e_run(local, hu, cd, ce, nc // 2, args.e2e_batches, 4096,
                                       args.window, ceil,
                                       flags=xdpgpu.CFG_DEFAULT | xdpgpu.CFG_HOST_COMPACT)
            e2e_compact_huge["workload"] = (e2e_compact["workload"] +
                                            ", UMEM in transparent huge pages (madvise; "
                                            f"THP {thp_mode()})")
            del hu, cu, cd, ce
            # the same with XDPGPU_CFG_UMEM_GATHER (a kernel reads each
            # frame's bytes through the UMEM's GPU mapping), in a child
            # process: the one kernel that reads host memory (DESIGN.md
            # §5.3) cannot take this line down with it
            e2e_gather = gather_leg(nc, args.e2e_batches, ceil)
            e2e_gather["workload"] = e2e_chunked["workload"] + ", XDPGPU_CFG_UMEM_GATHER"

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(umem, descs, xdpgpu.CFG_DEFAULT, xdpgpu.TUPLE_V4)

    if rank == 0:
        traffic, traffic_src = pmc_traffic(n, args.size)
        kernel_frac = BYTES_PER_FRAME * n / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS
        line = {
            "metric": METRIC,
            "value": round(mpps, 1),
            "unit": "Mpps",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": f"config2: {n} x {args.size}B IPv4/UDP frames per GPU, "
                                   "packed 64B-stride UMEM, 1% bad L3 / 1% bad L4 / "
                                   "0.5% malformed / 0.1% ARP / 0.1% NDP",
                       "frames_per_gpu": n, "frame_size": args.size,
                       "header_window": args.window or (128 if args.size >= 128 else 64),
                       "parallelism": f"shard{world}",
                       "in_flight": "2 launches (xdpgpu_submit_dev, two slots)",
                       **({"rehearsal": "ranks sharing GPUs, gloo"} if rehearse else {})},
            "gbps": round(gbps, 1),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         # algorithmic bytes of a launch over the timed
                         # launches' GPU span a step (events at the two ends
                         # of the K timed launches; the slowest rank)
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "timed_span_ms_per_launch": span_step,
                         # the same bytes over the timed wall time per step
                         # (host clock around the K launches, the driver's)
                         "frac_wall": round(BYTES_PER_FRAME * n * args.steps / wall_max / 1e9 /
                                            HBM_PEAK_GBS, 4),
                         # and over the kernel's own duration, one launch at
                         # a time between its event pair (what rocprofv3
                         # reports for those launches)
                         "frac_kernel": round(kernel_frac, 4),
                         "traffic": traffic,
                         "traffic_source": traffic_src,
                         "kernels": "+".join(RX_KERNELS),
                         "kernel_ms": kt_round(kt),
                         "bytes_per_frame": BYTES_PER_FRAME,
                         "algorithmic_bytes_per_launch": BYTES_PER_FRAME * n},
            "per_rank": per_rank,
            "devices": {"pci_bus_ids": [d["pci_bus_id"] for d in idents],
                        "name": ident["name"], "rccl": ident["rccl"],
                        "backend": ("gloo" if rehearse else "nccl") if world > 1 else None},
            "cpu_baseline": cpu,
            "verdicts_ok": all_ok,
        }
        line.update(secondary)
        if e2e:
            line["e2e_host_path"] = e2e
        if e2e_chunked:
            line["e2e_host_path_chunked"] = e2e_chunked
        if e2e_compact:
            line["e2e_host_path_chunked_compact"] = e2e_compact
        if e2e_compact_huge:
            line["e2e_host_path_chunked_compact_huge"] = e2e_compact_huge
        if e2e_gather:
            line["e2e_host_path_chunked_gather"] = e2e_gather
        print(json.dumps(line), flush=True)
    ctx.close()
    tctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
