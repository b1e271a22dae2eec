#!/usr/bin/env python3
# SPDX-License-Identifier: GPL-2.0
"""Diagnostic (not a test): per-wave timeline of the double-buffered RX
kernel from a stamps build (XDPGPU_LIB = build/stamps/libxdpgpu.so,
tools/dbg_build.sh stamps) on the config-2 pool: wave start / loop end /
end spreads overall and per XCD (blocks go round-robin to the 8 XCDs)."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "bpf-examples_amd"))
import torch  # noqa: E402
import xdpgpu  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16 << 20
tune = int(sys.argv[2], 0) if len(sys.argv) > 2 else 0
kind = int(sys.argv[3]) if len(sys.argv) > 3 else xdpgpu.POOL_UDP4
fmt = int(sys.argv[4]) if len(sys.argv) > 4 else xdpgpu.TUPLE_V4
lib = xdpgpu.load_library()
lib.xdpgpu_stamps_read.argtypes = [C.c_void_p]
# STAMPS_SIZE / STAMPS_ECHO_PPM: the echo leg's pool (bench.py echo_run:
# 128-byte frames, ICMPv6 echo requests answered, XDPGPU_CFG_ICMP6_ECHO)
size = int(os.environ.get("STAMPS_SIZE", "64"))
echo_ppm = int(os.environ.get("STAMPS_ECHO_PPM", "0"))
kw = {"ppm_echo6": echo_ppm} if echo_ppm else {}
seed = 0x5EED0042 if echo_ppm else 0x5EED0002 if kind == 0 else 0x5EED0003
umem, descs, _ = xdpgpu.pool_generate(n, kind, size, seed, **kw)
flags = xdpgpu.CFG_DEFAULT | (xdpgpu.CFG_ICMP6_ECHO if echo_ppm else 0)
dev = torch.device("cuda:0")
d_umem = torch.zeros(umem.nbytes + 64, dtype=torch.uint8, device=dev)
d_umem[: umem.nbytes].copy_(torch.from_numpy(umem))
d_desc = torch.from_numpy(descs.view(np.uint8)).to(dev)
d_v = torch.empty(n, dtype=torch.uint8, device=dev)
d_res = torch.empty(n * 16, dtype=torch.uint8, device=dev)
d_tup = torch.empty(n * 44, dtype=torch.uint8, device=dev)
# STAMPS_WINDOW: the header window (64, 128, 0 = the library's choice)
ctx = xdpgpu.XdpGpu(0, flags, 0, fmt, int(os.environ.get("STAMPS_WINDOW", "64")), tune=tune)
st = np.zeros(8 * 8192, np.uint64)
reps = int(os.environ.get("STAMPS_REPS", "6"))
per_rep = []   # per launch: each XCC's median and last loop end (us)
for rep in range(reps):
    st[:] = 0
    if echo_ppm:   # the responder rewrote the requests: restore them
        d_umem[: umem.nbytes].copy_(torch.from_numpy(umem))
        torch.cuda.synchronize()
    ctx.process_dev(d_umem, umem.nbytes, d_desc, n, d_v, d_res, d_tup)
    torch.cuda.synchronize()
    lib.xdpgpu_stamps_read(st.ctypes.data)
    r4 = st.reshape(-1, 8)
    lv = r4[:, 0] > 0
    rs = r4[lv][:, [0, 1, 2]].astype(np.int64)
    rt = (rs - rs[:, 0].min()) / 100.0
    xc = ((r4[lv, 3] >> 32) & 0xF).astype(int)
    per_rep.append({"xcc_loop_end_median": [round(float(np.median(rt[xc == k, 1])), 1)
                                            for k in range(8)],
                    "xcc_loop_end_max": [round(float(rt[xc == k, 1].max()), 1)
                                         for k in range(8)],
                    "end_max": round(float(rt[:, 2].max()), 1)})
s4 = st.reshape(-1, 8)
live = s4[:, 0] > 0
hw = s4[live, 3]
s = s4[live][:, [0, 1, 2]].astype(np.int64)
t0 = s[:, 0].min()
us = (s - t0) / 100.0            # 100 MHz ticks -> us
ph = s4[live][:, 4:8].astype(np.int64) / 100.0   # tail time per batch kind
waves = np.nonzero(live)[0]
# blocks of the double-buffered kernel (15 waves each) go round-robin to
# the 8 XCDs
xcd = (waves // 15) % 8


def pct(a):
    return [round(float(x), 1) for x in np.percentile(a, [0, 10, 50, 90, 100])]


out = {"waves": int(live.sum()), "tail_us": pct(us[:, 2] - us[:, 1]),
       "tail_exception_us": pct(ph[:, 0]), "tail_bulk_us": pct(ph[:, 1]),
       "tail_payload_us": pct(ph[:, 2]), "tail_wait_us": pct(ph[:, 3]),
       "start_us": pct(us[:, 0]), "loop_end_us": pct(us[:, 1]),
       "end_us": pct(us[:, 2]), "loop_us": pct(us[:, 1] - us[:, 0])}
# its shared-tile heads (block b: head b mod 16)
blk = waves // 15
head = blk % 16
out["per_head_loop_end_median"] = [round(float(np.median(us[head == k, 1])), 1) for k in range(16)]
out["per_head_loop_end_max"] = [round(float(us[head == k, 1].max()), 1) for k in range(16)]
out["per_xcd_loop_end_median"] = [round(float(np.median(us[xcd == k, 1])), 1) for k in range(8)]
out["per_xcd_loop_end_max"] = [round(float(us[xcd == k, 1].max()), 1) for k in range(8)]
# where each wave ran: HW_ID (wave 3:0, simd 5:4, cu 11:8, sh 12, se 15:13),
# XCC_ID in the high word
lo = (hw & 0xFFFFFFFF).astype(np.int64)
cu = ((hw >> 32) & 0xF).astype(np.int64) * 4096 + ((lo >> 8) & 0xFF)
simd = (lo >> 4) & 3
out["xcc_ids"] = sorted(set(((hw >> 32) & 0xF).astype(int).tolist()))
cus = np.unique(cu)
out["cus"] = len(cus)
spread, means, rank_corr = [], [], []
for c in cus:
    m = cu == c
    le = us[m, 1]
    spread.append(le.max() - le.min())
    means.append(le.mean())
    # launch order within the CU (block index) against loop end
    order = np.argsort(np.argsort(waves[m]))
    rk = np.argsort(np.argsort(le))
    if m.sum() > 2:
        rank_corr.append(np.corrcoef(order, rk)[0, 1])
out["waves_per_cu"] = pct(np.array([int((cu == c).sum()) for c in cus]))
out["within_cu_spread_us"] = pct(np.array(spread))
# where the launch ends: each CU's last wave against its mean, and the CUs'
# last waves against each other (the tail phase's imbalance)
out["within_cu_end_spread_us"] = pct(np.array([np.ptp(us[cu == c, 2]) for c in cus]))
out["cu_max_end_us"] = pct(np.array([us[cu == c, 2].max() for c in cus]))
out["cu_mean_end_us"] = pct(np.array([us[cu == c, 2].mean() for c in cus]))
out["cu_mean_loop_end_us"] = pct(np.array(means))
out["rank_corr_launch_order_vs_end"] = round(float(np.mean(rank_corr)), 3)
# per SIMD slot: the waves of one SIMD ranked by launch order
ends_by_age = [[] for _ in range(8)]
for c in cus:
    for sd in range(4):
        m = (cu == c) & (simd == sd)
        idx = np.argsort(waves[m])
        for r, v in enumerate(us[m, 1][idx]):
            if r < 8:
                ends_by_age[r].append(v)
out["loop_end_by_age_on_simd"] = [round(float(np.median(x)), 1) if x else None
                                  for x in ends_by_age]
out["per_launch"] = per_rep
print(json.dumps(out))
