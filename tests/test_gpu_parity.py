# SPDX-License-Identifier: GPL-2.0
"""GPU parity: the HIP path (through the C ABI) against the committed golden
vectors and the oracle, bit-exact, on the same inputs.  Runs on the MI355X
box (`pytest -m gpu`)."""
import numpy as np
import pytest

import oracle
import xdpgpu

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

CFG_FLAGS = {"verify": 0x5, "echo_net": 0x7, "noverify": 0x4}


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    assert xdpgpu.device_count() > 0
    return torch.device("cuda:0")


def to_dev(a: np.ndarray, pad: int = 64):
    t = torch.zeros(a.nbytes + pad, dtype=torch.uint8, device="cuda:0")
    t[: a.nbytes].copy_(torch.from_numpy(a.view(np.uint8).reshape(-1)))
    return t


# kernel variants (cfg.tune): default (one fused launch); every frame through
# the exception pipeline of the launch's tail (bit 9); the same with the
# exception pass keeping its payload sums (bit 8); no shared tiles (bit 21);
# shared tiles without the partner head (bit 28)
TUNES = [0, 512, 512 | 256, 1 << 21, 1 << 28]
# (cfg.tune, cfg.window): every tune with 64-byte windows; the 128-byte
# window kernel (a long frame starting a 128-byte line has its bytes
# [64, 128) staged too) with the default, all-exception, no-shared-tile and
# no-partner tunes
VARIANTS = [(t, 64) for t in TUNES] + [(0, 128), (512, 128), (1 << 21, 128), (1 << 28, 128)]
SHORT_VARIANTS = [(0, 64), (512, 64), (1 << 21, 64), (0, 128), (512, 128)]


def run_dev(umem, descs, flags=0x5, initval=0, fmt=1, window=64, tune=0):
    """Device-resident path; returns verdict, res, tuples, umem after, stats."""
    n = len(descs)
    ctx = xdpgpu.XdpGpu(0, flags | xdpgpu.CFG_STATS, initval, fmt, window, tune=tune)
    d_umem = to_dev(umem)
    d_desc = to_dev(np.ascontiguousarray(descs, xdpgpu.DESC_DTYPE), 16)
    d_v = torch.full((max(n, 1),), 0xEE, dtype=torch.uint8, device="cuda:0")
    d_res = torch.full((max(n, 1) * 16,), 0xEE, dtype=torch.uint8, device="cuda:0")
    tb = xdpgpu.TUPLE_BYTES[fmt]
    d_tup = torch.full((max(n * tb, 1),), 0xEE, dtype=torch.uint8, device="cuda:0") \
        if tb else None
    s = torch.cuda.current_stream()
    ctx.process_dev(d_umem, umem.nbytes, d_desc, n, d_v, d_res, d_tup, stream=s)
    torch.cuda.synchronize()
    st = ctx.stats()
    ctx.close()
    v = d_v.cpu().numpy()[:n]
    res = d_res.cpu().numpy()[: n * 16].view(xdpgpu.RESULT_DTYPE)
    tup = d_tup.cpu().numpy()[: n * tb] if tb else None
    um = d_umem.cpu().numpy()[: umem.nbytes]
    return v, res, tup, um, st


def assert_same(got, want, what):
    gv, gres, gtup, gum = got
    wv, wres, wtup, wum = want
    bad = np.nonzero(gv != wv)[0]
    assert len(bad) == 0, f"{what}: verdict mismatch at {bad[:8]}: {gv[bad[:8]]} vs {wv[bad[:8]]}"
    gr, wr = gres.view(np.uint8).reshape(-1, 16), wres.view(np.uint8).reshape(-1, 16)
    bad = np.nonzero((gr != wr).any(1))[0]
    assert len(bad) == 0, f"{what}: result mismatch at {bad[:8]}:\n{gres[bad[:4]]}\n{wres[bad[:4]]}"
    if wtup is not None:
        tb = len(wtup) // max(len(wv), 1)
        gt, wt = gtup.reshape(-1, tb), wtup.reshape(-1, tb)
        bad = np.nonzero((gt != wt).any(1))[0]
        assert len(bad) == 0, f"{what}: tuple mismatch at {bad[:8]}"
    if gum is not None and wum is not None:
        assert np.array_equal(gum, wum), f"{what}: UMEM after differs"


def oracle_stats_match(st, ost):
    assert st["frames"] == ost["frames"] and st["bytes"] == ost["bytes"]
    assert [st["verdict"][n] for n in xdpgpu.VERDICT_NAMES] == ost["verdict"]
    for k in ("l3_bad", "l4_bad", "l4_absent", "frag"):
        assert st[k] == ost[k], k


# ---------------------------------------------------------------- golden
@pytest.mark.parametrize("tune,window", VARIANTS)
@pytest.mark.parametrize("cfg", ["verify", "echo_net", "noverify"])
def test_golden_fixtures_device(dev, golden, cfg, tune, window):
    fx, meta = golden
    flags, iv, fmt = meta["cfgs"][cfg]
    descs = fx["descs"].view(xdpgpu.DESC_DTYPE)
    v, res, tup, um, st = run_dev(fx["umem"], descs, flags, iv, fmt, window, tune)
    want = (fx[f"{cfg}_verdict"], fx[f"{cfg}_res"].view(xdpgpu.RESULT_DTYPE),
            fx[f"{cfg}_tup"], fx[f"{cfg}_umem_after"])
    assert_same((v, res, tup, um), want, f"golden/{cfg}")
    ws = fx[f"{cfg}_stats"]
    assert st["frames"] == ws[0] and st["bytes"] == ws[1]
    assert [st["verdict"][n] for n in xdpgpu.VERDICT_NAMES] == list(ws[2:7])
    assert [st["l3_bad"], st["l4_bad"], st["l4_absent"], st["frag"]] == list(ws[7:11])


@pytest.mark.parametrize("cfg", ["verify", "echo_net"])
def test_golden_fixtures_host_path(dev, golden, cfg):
    """xdpgpu_process on host buffers (pinned UMEM, span copy, D2H)."""
    fx, meta = golden
    flags, iv, fmt = meta["cfgs"][cfg]
    umem = fx["umem"].copy()
    descs = fx["descs"].view(xdpgpu.DESC_DTYPE).copy()
    with xdpgpu.XdpGpu(0, flags, iv, fmt) as ctx:
        ctx.register_umem(umem)
        v, res, tup = ctx.process(descs)
    assert_same((v, res, tup.view(np.uint8).reshape(-1), umem),
                (fx[f"{cfg}_verdict"], fx[f"{cfg}_res"].view(xdpgpu.RESULT_DTYPE),
                 fx[f"{cfg}_tup"], fx[f"{cfg}_umem_after"]), f"host/{cfg}")


# ---------------------------------------------------------------- pools
POOLS = [
    ("udp4_64", xdpgpu.POOL_UDP4, 64, 0x5EED0002, 1 << 20, {}),
    ("udp4_1500", xdpgpu.POOL_UDP4, 1500, 0x5EED0002, 100000, {}),
    ("imix", xdpgpu.POOL_IMIX, 64, 0x5EED0003, 300000, {}),
    ("udp4_64_odd_addr", xdpgpu.POOL_UDP4, 64, 7, 100000, dict(headroom=1, stride=128)),
    ("imix_4mod16", xdpgpu.POOL_IMIX, 64, 8, 50000, dict(headroom=4, stride=2048)),
    ("echo6", xdpgpu.POOL_UDP4, 128, 9, 100000, dict(ppm_echo6=200000)),
]


@pytest.mark.parametrize("tune,window", VARIANTS)
@pytest.mark.parametrize("name,kind,size,seed,n,kw", POOLS, ids=[p[0] for p in POOLS])
def test_pool_vs_oracle(dev, name, kind, size, seed, n, kw, tune, window):
    umem, descs, expect = xdpgpu.pool_generate(n, kind, size, seed, **kw)
    for flags, iv, fmt in ((0x5, 0, 1), (0x7, 0x9E3779B9, 2)):
        ou = umem.copy()
        ov, ores, otup, ost = oracle.process(ou, descs, flags, iv, fmt)
        v, res, tup, um, st = run_dev(umem, descs, flags, iv, fmt, window, tune)
        assert_same((v, res, tup, um), (ov, ores, otup, ou), f"{name}/{flags:#x}")
        oracle_stats_match(st, ost)
        if flags == 0x5:
            np.testing.assert_array_equal(v, expect)


def bulk_frames(seed: int, n: int, long_every: int = 3, aligned: bool = True):
    """Fast-shape IPv4 UDP/TCP/ICMP frames of every length class around and past
    the 64-byte header window (0..2 VLAN tags, odd lengths, trailing pad,
    bad and absent checksums), 16-byte aligned with random gaps; the last
    frame ends at the UMEM end with an odd UDP length (over-read past the
    UMEM reads as zero).  Every long_every-th frame has up to 2960 payload
    bytes, the rest under 60 (long_every 0: none long, so that whole bulk
    batches have ranges within 64 bytes); aligned False puts frames at any
    byte offset (exception frames, whose payload sums the bulk pass adds
    from unaligned ranges)."""
    import frames as F
    rng = np.random.default_rng(seed)
    blobs = []
    for k in range(n):
        tags = [(0x8100, 5)] * int(rng.integers(0, 3))
        plen = int(rng.integers(0, 60)) if not long_every or k % long_every \
            else int(rng.integers(0, 2960))
        pay = rng.integers(0, 256, plen, dtype=np.uint8).tobytes()
        if rng.random() < 0.5 or k == n - 1:
            seg = F.udp(int(rng.integers(1, 65536)), 53, pay)
            fr = F.v4_frame(17, seg, tags=tags)
            if rng.random() < 0.05:
                fr = fr[:-len(seg)] + F.set_csum(seg, 6, 0)
        elif rng.random() < 0.2:
            # IPv4 ICMP: the fast shape of the network_tuple builds (no
            # pseudo header, no over-read byte)
            fr = F.v4_frame(1, F.icmp(8, 0, b"\x12\x34\x00\x01" + pay), tags=tags)
        else:
            fr = F.v4_frame(6, F.tcp(int(rng.integers(1, 65536)), 80, pay,
                                     doff=int(rng.integers(5, 9))), tags=tags)
        if rng.random() < 0.1 and plen:
            b = bytearray(fr)
            b[-1 - int(rng.integers(0, plen))] ^= 0x5A
            fr = bytes(b)
        if rng.random() < 0.1 and k != n - 1:
            fr += rng.integers(0, 256, int(rng.integers(1, 9)), dtype=np.uint8).tobytes()
        blobs.append(fr)
    if len(blobs[-1]) % 2 == 0:        # odd UDP length for the last frame
        seg = F.udp(7, 53, b"\x11" * 31)
        blobs[-1] = F.v4_frame(17, seg)
    offs, o = [], 0
    for fr in blobs:
        o += 16 * int(rng.integers(0, 4)) if aligned else int(rng.integers(0, 40))
        offs.append(o)
        o = (o + len(fr) + 15) & ~15 if aligned else o + len(fr)
    size = offs[-1] + len(blobs[-1])
    umem = np.zeros(size, np.uint8)
    for off, fr in zip(offs, blobs):
        umem[off:off + len(fr)] = np.frombuffer(fr, np.uint8)
    descs = np.zeros(n, xdpgpu.DESC_DTYPE)
    descs["addr"] = offs
    descs["len"] = [len(fr) for fr in blobs]
    return umem, descs


@pytest.mark.parametrize("tune,window", VARIANTS)
@pytest.mark.parametrize("aligned", [True, False])
def test_bulk_lengths_vs_oracle(dev, tune, window, aligned):
    """The bulk path (checksum ranges past the window) and its boundaries;
    long ranges start at every 16-byte (aligned: fast-shape frames) or byte
    (exception frames) offset in their first 128-byte line, which the bulk
    pass streams from (XDP_TAIL_LINE_AL)."""
    umem, descs = bulk_frames(21 if aligned else 22, 3000, aligned=aligned)
    for flags, iv, fmt in ((0x5, 0, 1), (0x4, 0x12345, 2)):
        ov, ores, otup, ost = oracle.process(umem.copy(), descs, flags, iv, fmt)
        v, res, tup, um, st = run_dev(umem, descs, flags, iv, fmt, window, tune)
        assert_same((v, res, tup, None), (ov, ores, otup, None), f"bulk/{aligned}/{flags:#x}")
        oracle_stats_match(st, ost)
        if flags == 0x5:
            assert (ov == xdpgpu.REDIRECT).sum() > 2000 and (ov == xdpgpu.DROP).sum() > 100


def shared_line_frames(seed: int, n: int):
    """Frames laid so that each range ends in the first half of the line
    the next frame starts 64 bytes into (XDP_TAIL_SHARE: the next lane's
    window holds those bytes): IPv4 UDP (odd and even lengths, the odd
    ones' over-read byte the last byte before the next frame), TCP, ICMP,
    0..2 tags, and IPv6 UDP/TCP/ICMPv6 behind 0..1 tag starting a line;
    the range ending 1..64 bytes before the next frame, some with pad or
    a gap, some starting 16 bytes off a 64-byte boundary (not taken), a
    tenth with a corrupted payload byte."""
    import frames as F
    rng = np.random.default_rng(seed)
    blobs, offs, o = [], [], 0
    for k in range(n):
        v6 = rng.random() < 0.3
        tags = [(0x8100, 5)] * int(rng.integers(0, 2 if v6 else 3))
        # frame start: a line start (IPv6: its window's second half staged)
        # or 64 bytes into one; now and then 16 bytes off
        o = (o + 127) & ~127 if v6 else (o + 63) & ~63
        if not v6 and rng.random() < 0.1:
            o += 16
        start = o
        # the range end: 1..64 bytes into the line after a line start 64
        # bytes before the next frame
        hdr = 14 + 4 * len(tags) + (40 if v6 else 20)
        lines = int(rng.integers(1, 12))
        nxt = ((start + hdr + 8 + 127) // 128 + lines) * 128 + 64
        end = nxt - int(rng.integers(0, 64))           # range end, exclusive
        kind = int(rng.integers(0, 3))
        if v6:
            plen = end - start - hdr - 8
            pay = rng.integers(0, 256, max(plen, 0), dtype=np.uint8).tobytes()
            seg = (F.udp(4000 + k, 53, pay) if kind == 0 else
                   F.tcp(4000 + k, 80, pay[8:] if len(pay) >= 12 else pay) if kind == 1 else
                   F.icmp(128, 0, b"\x12\x34\x00\x01" + pay))
            fr = F.v6_frame({0: 17, 1: 6, 2: 58}[kind], seg, tags=tags)
        else:
            proto = {0: 17, 1: 6, 2: 1}[kind]
            plen = end - start - hdr - 8 - (1 if proto == 17 and rng.random() < 0.5 else 0)
            pay = rng.integers(0, 256, max(plen, 0), dtype=np.uint8).tobytes()
            seg = (F.udp(4000 + k, 53, pay) if proto == 17 else
                   F.tcp(4000 + k, 80, pay[12:] if len(pay) >= 12 else pay) if proto == 6 else
                   F.icmp(8, 0, b"\x12\x34\x00\x01" + pay))
            fr = F.v4_frame(proto, seg, tags=tags)
        if rng.random() < 0.1:
            b = bytearray(fr)
            b[-1 - int(rng.integers(0, 8))] ^= 0x5A
            fr = bytes(b)
        if rng.random() < 0.2:
            fr += rng.integers(0, 256, int(rng.integers(1, 9)), dtype=np.uint8).tobytes()
        blobs.append(fr)
        offs.append(start)
        o = max(start + len(fr), nxt - (0 if rng.random() < 0.8 else 64))
    size = offs[-1] + len(blobs[-1]) + 1
    umem = np.zeros(size, np.uint8)
    for off, fr in zip(offs, blobs):
        umem[off:off + len(fr)] = np.frombuffer(fr, np.uint8)
    # bytes between frames: not zero, so that a wrongly masked half-line
    # changes the sum
    gap = np.ones(size, bool)
    for off, fr in zip(offs, blobs):
        gap[off:off + len(fr)] = False
    umem[gap] = rng.integers(1, 256, int(gap.sum()), dtype=np.uint8)
    descs = np.zeros(n, xdpgpu.DESC_DTYPE)
    descs["addr"] = offs
    descs["len"] = [len(fr) for fr in blobs]
    return umem, descs


@pytest.mark.parametrize("tune,window", [(0, 64), (0, 128), (512, 128), (1 << 21, 128)])
def test_shared_line_vs_oracle(dev, tune, window):
    """A frame whose range ends in the first half of the line the next
    frame starts 64 bytes into: the next lane sums those bytes for it and
    the bulk pass stops at the line start (XDP_TAIL_SHARE, 128-byte
    windows)."""
    umem, descs = shared_line_frames(31, 4000)
    for flags, iv, fmt in ((0x5, 0, 1), (0x4, 0x12345, 2), (0x5, 7, 0)):
        ov, ores, otup, ost = oracle.process(umem.copy(), descs, flags, iv, fmt)
        v, res, tup, um, st = run_dev(umem, descs, flags, iv, fmt, window, tune)
        assert_same((v, res, tup, None), (ov, ores, otup, None), f"shared/{flags:#x}")
        oracle_stats_match(st, ost)
        if flags == 0x5 and fmt == 1:
            # (odd lengths over-read the next, non-zero byte: DROP, with
            # the record's sum still compared)
            assert (ov == xdpgpu.REDIRECT).sum() > 2000 and (ov == xdpgpu.DROP).sum() > 100


@pytest.mark.parametrize("tune,window", SHORT_VARIANTS)
@pytest.mark.parametrize("aligned", [True, False])
def test_short_bulk_vs_oracle(dev, tune, window, aligned):
    """Bulk batches whose ranges all end within 64 bytes of the window
    (stream_short) and batches just past that, fast-shape (aligned) and
    exception (unaligned) frames."""
    umem, descs = bulk_frames(23 + aligned, 6000, long_every=0, aligned=aligned)
    for flags, iv, fmt in ((0x5, 0, 1), (0x4, 0x12345, 2), (0x7, 9, 0)):
        ou = umem.copy()
        ov, ores, otup, ost = oracle.process(ou, descs, flags, iv, fmt)
        v, res, tup, um, st = run_dev(umem, descs, flags, iv, fmt, window, tune)
        assert_same((v, res, tup, um), (ov, ores, otup, ou), f"short/{aligned}/{flags:#x}")
        oracle_stats_match(st, ost)
        if flags == 0x5:
            assert (ov == xdpgpu.REDIRECT).sum() > 4000 and (ov == xdpgpu.DROP).sum() > 200


@pytest.mark.parametrize("window", [64, 128])
def test_unaligned_encoded_descriptors(dev, window):
    """Unaligned-chunk addresses (offset << 48 | base, if_xdp.h:104-106)."""
    umem, descs, _ = xdpgpu.pool_generate(50000, xdpgpu.POOL_IMIX, 64, 11)
    enc = descs.copy()
    base = enc["addr"] & ~np.uint64(0xFFF)
    enc["addr"] = ((enc["addr"] - base) << np.uint64(48)) | base
    ov, ores, otup, _ = oracle.process(umem.copy(), descs, 0x5, 0, 1)
    v, res, tup, um, _ = run_dev(umem, enc, 0x5, 0, 1, window)
    assert_same((v, res, tup, None), (ov, ores, otup, None), "encoded")


def test_full_size_config2(dev):
    """BASELINE config 2 at full size: 16 M x 64 B.  Bit-exact against the
    oracle for every frame, and the generator's intended verdicts."""
    n = 16 << 20
    umem, descs, expect = xdpgpu.pool_generate(n, xdpgpu.POOL_UDP4, 64, 0x5EED0002)
    v, res, tup, _, st = run_dev(umem, descs, 0x5, 0, 1)
    np.testing.assert_array_equal(v, expect)
    ov, ores, otup, ost = oracle.process(umem, descs, 0x5, 0, 1)
    assert_same((v, res, tup, None), (ov, ores, otup, None), "config2-16M")
    oracle_stats_match(st, ost)


def test_full_size_config3(dev):
    """Config 3 at full size: 16 M IMIX frames (5.98 GB, 30 % IPv6, VLAN
    tags, the 44-byte network_tuple), as the bench leg runs it.  Bit-exact
    against the oracle for every frame, and the generator's verdicts."""
    n = 16 << 20
    umem, descs, expect = xdpgpu.pool_generate(n, xdpgpu.POOL_IMIX, 64, 0x5EED0003)
    v, res, tup, _, st = run_dev(umem, descs, 0x5, 0, 2, 0)     # window: automatic (128)
    np.testing.assert_array_equal(v, expect)
    ov, ores, otup, ost = oracle.process(umem, descs, 0x5, 0, 2)
    assert_same((v, res, tup, None), (ov, ores, otup, None), "config3-16M")
    oracle_stats_match(st, ost)


def test_repeat_launches_identical(dev):
    """The HIP path against itself: one context, the same device batch
    launched back to back (the shared-tile counters alternate between their
    two sets, the tiles go to whichever CU claims them first) and on a
    second stream, outputs identical byte for byte every time."""
    umem, descs, _ = xdpgpu.pool_generate(1 << 20, xdpgpu.POOL_IMIX, 64, 0x5EED0013)
    ctx = xdpgpu.XdpGpu(0, 0x5, 0x1234, 2, 64)
    d_umem, d_desc = to_dev(umem), to_dev(np.ascontiguousarray(descs, xdpgpu.DESC_DTYPE), 16)
    n = len(descs)
    outs = []
    s2 = torch.cuda.Stream()
    for k in range(6):
        d_v = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda:0")
        d_res = torch.full((n * 16,), 0xEE, dtype=torch.uint8, device="cuda:0")
        d_tup = torch.full((n * 44,), 0xEE, dtype=torch.uint8, device="cuda:0")
        torch.cuda.synchronize()
        stream = s2.cuda_stream if k >= 4 else None
        ctx.process_dev(d_umem, umem.nbytes, d_desc, n, d_v, d_res, d_tup, stream)
        ctx.sync(stream)
        outs.append((d_v.cpu().numpy(), d_res.cpu().numpy(), d_tup.cpu().numpy()))
    ctx.close()
    for k, o in enumerate(outs[1:], 1):
        for x, y, what in zip(outs[0], o, ("verdict", "record", "tuple")):
            assert np.array_equal(x, y), f"launch {k}: {what} differs"


def test_submit_dev_two_slots_vs_oracle(dev):
    """xdpgpu_submit_dev, the device-resident RX loop with two batches in
    flight (bench.py's timed loop): consecutive batches of one pool dealt
    to the two slots, each into its own outputs, launched without a host
    wait between them so that they overlap on the GPU; every frame's
    verdict, record and tuple, and the counters, against the oracle.  Then
    the same batch on both slots at once, byte-identical; a slot with a
    host batch in flight refuses a device batch (-EBUSY)."""
    umem, descs, _ = xdpgpu.pool_generate(1 << 20, xdpgpu.POOL_IMIX, 64, 0x5EED0014)
    descs = np.ascontiguousarray(descs, xdpgpu.DESC_DTYPE)
    ov, ores, otup, ost = oracle.process(umem.copy(), descs, 0x5, 0, 2)
    n = len(descs)
    B = n // 8
    d_umem, d_desc = to_dev(umem), to_dev(descs, 16)
    d_v = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda:0")
    d_res = torch.full((n * 16,), 0xEE, dtype=torch.uint8, device="cuda:0")
    d_tup = torch.full((n * 44,), 0xEE, dtype=torch.uint8, device="cuda:0")
    with xdpgpu.XdpGpu(0, 0x5, 0, 2, 0) as ctx:
        assert ctx.slot_stream(0) and ctx.slot_stream(1)
        assert ctx.slot_stream(0) != ctx.slot_stream(1)
        torch.cuda.synchronize()
        for k in range(8):
            lo = k * B
            ctx.submit_dev(k & 1, d_umem, umem.nbytes, d_desc[lo * 16:], B, d_v[lo:],
                           d_res[lo * 16:], d_tup[lo * 44:])
        ctx.wait(0)
        ctx.wait(1)
        st = ctx.stats()
        np.testing.assert_array_equal(d_v.cpu().numpy(), ov)
        assert d_res.cpu().numpy().tobytes() == ores.tobytes()
        assert d_tup.cpu().numpy().tobytes() == otup.tobytes()
        assert st["frames"] == ost["frames"] == n
        assert [st["verdict"][x] for x in xdpgpu.VERDICT_NAMES] == ost["verdict"]
        # one batch on both slots at once, each into its own outputs
        outs = [(torch.empty(n, dtype=torch.uint8, device="cuda:0"),
                 torch.empty(n * 16, dtype=torch.uint8, device="cuda:0"),
                 torch.empty(n * 44, dtype=torch.uint8, device="cuda:0")) for _ in range(2)]
        for k in range(6):
            ctx.submit_dev(k & 1, d_umem, umem.nbytes, d_desc, n, *outs[k & 1])
        ctx.sync()
        for v, r, t in outs:
            np.testing.assert_array_equal(v.cpu().numpy(), ov)
            assert r.cpu().numpy().tobytes() == ores.tobytes()
            assert t.cpu().numpy().tobytes() == otup.tobytes()
        # a host batch in flight on slot 1: its device batch is refused
        ctx.register_umem(umem)
        hv = np.zeros(1024, np.uint8)
        ctx.submit(1, descs[:1024], hv)
        with pytest.raises(xdpgpu.XdpGpuError, match="EBUSY|busy|in flight"):
            ctx.submit_dev(1, d_umem, umem.nbytes, d_desc, n, *outs[1])
        ctx.wait(1)
        np.testing.assert_array_equal(hv, ov[:1024])


def test_empty_batch(dev):
    umem, descs, _ = xdpgpu.pool_generate(4, xdpgpu.POOL_UDP4, 64, 1)
    v, res, tup, um, st = run_dev(umem, descs[:0], 0x5, 0, 1)
    assert len(v) == 0 and st["frames"] == 0


def test_host_double_buffer(dev):
    """xdpgpu_submit/xdpgpu_wait on both slots, batches of an RX loop."""
    umem, descs, expect = xdpgpu.pool_generate(200000, xdpgpu.POOL_IMIX, 64, 12)
    ov, ores, otup, _ = oracle.process(umem.copy(), descs, 0x5, 0, 1)
    B = 4096
    with xdpgpu.XdpGpu(0, 0x5, 0, 1, max_batch=B) as ctx:
        ctx.register_umem(umem)
        v = np.zeros(len(descs), np.uint8)
        res = np.zeros(len(descs), xdpgpu.RESULT_DTYPE)
        tup = np.zeros(len(descs), xdpgpu.TUPLE4_DTYPE)
        pending = [None, None]
        for k, lo in enumerate(range(0, len(descs), B)):
            slot = k & 1
            if pending[slot] is not None:
                ctx.wait(slot)
            hi = min(lo + B, len(descs))
            d = np.ascontiguousarray(descs[lo:hi])
            pending[slot] = d
            ctx.submit(slot, d, v[lo:hi], res[lo:hi], tup[lo:hi])
        ctx.wait(0)
        ctx.wait(1)
        st = ctx.stats()
    assert_same((v, res, tup.view(np.uint8).reshape(-1), None),
                (ov, ores, otup, None), "double-buffer")
    assert st["frames"] == len(descs)


# ---------------------------------------------------------------- primitives
def test_jhash_primitive_vectors(dev):
    import os
    vec = np.load(os.path.join(os.path.dirname(__file__), "golden", "jhash_vectors.npz"))
    keys, klen, iv, want = vec["keys"], vec["klen"], vec["initval"], vec["jhash"]
    ctx = xdpgpu.XdpGpu(0)
    d_keys = to_dev(np.ascontiguousarray(keys))
    out = torch.zeros(len(klen), dtype=torch.int32, device="cuda:0")
    for L in np.unique(klen):
        idx = np.nonzero(klen == L)[0]
        for k in idx:
            ctx.jhash_dev(d_keys.data_ptr() + int(k) * 64, int(L), 64, 1, int(iv[k]),
                          out.data_ptr() + 4 * int(k))
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(got, want)
    ctx.close()


def test_jhash_word_primitive_vectors(dev):
    """jhash2 over 0..16 words with per-key initvals, and jhash_1word /
    2words / 3words: reference-generated vectors (make_golden.py)."""
    import os
    vec = np.load(os.path.join(os.path.dirname(__file__), "golden", "jhash_vectors.npz"))
    keys = np.ascontiguousarray(vec["keys"][:500]).view(np.uint32)      # 16 words each
    wl, iv = vec["wlen"], vec["initval"][:500]
    ctx = xdpgpu.XdpGpu(0)
    d_keys = to_dev(keys)
    out = torch.zeros(500, dtype=torch.int32, device="cuda:0")
    for k in range(500):
        ctx.jhash2_dev(d_keys.data_ptr() + 64 * k, int(wl[k]), 16, 1, int(iv[k]),
                       out.data_ptr() + 4 * k)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), vec["jhash2"])
    # one launch of 500 keys of one length: stride and batch indexing
    for L in (0, 1, 11, 16):
        ctx.jhash2_dev(d_keys, L, 16, 500, 0x9E3779B9, out)
        torch.cuda.synchronize()
        want = [oracle.lib().oracle_jhash2(keys[k].tobytes(), L, 0x9E3779B9)
                for k in range(500)]
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32),
                                      np.array(want, np.uint32))
    w3 = np.ascontiguousarray(vec["words3"])
    d_w3 = to_dev(w3)
    for nw, key in ((3, "jhash_3words"), (2, "jhash_2words"), (1, "jhash_1word")):
        for k in range(500):
            ctx.jhash_nwords_dev(d_w3.data_ptr() + 12 * k, nw, 3, 1, int(iv[k]),
                                 out.data_ptr() + 4 * k)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), vec[key], err_msg=key)
    ctx.close()


def test_ip_fast_csum_primitive_vectors(dev):
    import os
    vec = np.load(os.path.join(os.path.dirname(__file__), "golden", "csum_vectors.npz"))
    hdrs = np.ascontiguousarray(vec["hdrs"])
    ctx = xdpgpu.XdpGpu(0)
    d = to_dev(hdrs)
    out = torch.zeros(len(hdrs), dtype=torch.int16, device="cuda:0")
    ctx.ip_fast_csum_dev(d, 60, len(hdrs), out)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint16), vec["ip_fast_csum"])
    ctx.close()


def icmp6_frames(seed: int, n: int):
    """Untagged ICMPv6 frames of every type class (NDP 133-137, echo
    request/reply, errors, unknown), lengths around and past the 64-byte
    window (odd ones too), some with bad checksums or a trailing pad, 16-byte
    aligned; and UDP/IPv6 frames beside them."""
    import frames as F
    rng = np.random.default_rng(seed)
    types = [1, 2, 3, 4, 128, 129, 130, 133, 134, 135, 136, 137, 143, 200]
    blobs = []
    for k in range(n):
        plen = int(rng.integers(0, 60)) if k % 3 else int(rng.integers(0, 1500))
        pay = rng.integers(0, 256, plen, dtype=np.uint8).tobytes()
        if k % 5 == 4:
            fr = F.v6_frame(17, F.udp(int(rng.integers(1, 65536)), 53, pay))
        else:
            typ = types[k % len(types)]
            fr = F.v6_frame(58, F.icmp(typ, int(rng.integers(0, 3)), b"\x00\x01\x00\x02" + pay))
        if rng.random() < 0.1:
            b = bytearray(fr)
            b[-1 - int(rng.integers(0, 8))] ^= 0x5A
            fr = bytes(b)
        if rng.random() < 0.1:
            fr += rng.integers(0, 256, int(rng.integers(1, 9)), dtype=np.uint8).tobytes()
        blobs.append(fr)
    offs, o = [], 0
    for fr in blobs:
        o += 16 * int(rng.integers(0, 3))
        offs.append(o)
        o = (o + len(fr) + 15) & ~15
    umem = np.zeros(o + 16, np.uint8)
    for off, fr in zip(offs, blobs):
        umem[off:off + len(fr)] = np.frombuffer(fr, np.uint8)
    descs = np.zeros(n, xdpgpu.DESC_DTYPE)
    descs["addr"] = offs
    descs["len"] = [len(fr) for fr in blobs]
    return umem, descs


def v6_late_frames(seed: int, n: int):
    """IPv6 frames behind 0, 1 or 2 VLAN tags (802.1Q / 802.1ad) with UDP,
    TCP or ICMPv6 and no extension header: the fast shape's "late" check
    words (TCP; UDP behind a tag; ICMPv6 behind two) and the shapes just
    outside it (UDP and TCP behind two tags).  TCP data offsets below 5,
    past the frame and past the payload length (parse_tcphdr: ABORTED);
    odd lengths, bad checksums, trailing pad, lengths from the smallest
    that parse to past 1500 B; 16-byte aligned, the last frame ending at
    the UMEM end."""
    import frames as F
    rng = np.random.default_rng(seed)
    blobs = []
    for k in range(n):
        tags = [[], [(0x8100, 7)], [(0x88A8, 3), (0x8100, 9)]][k % 3]
        kind = (k // 3) % 4
        plen = int(rng.integers(0, 40)) if k % 2 else int(rng.integers(0, 1600))
        pay = rng.integers(0, 256, plen, dtype=np.uint8).tobytes()
        pad = b""
        if kind == 0:
            fr = F.v6_frame(17, F.udp(int(rng.integers(1, 65536)), 53, pay), tags=tags)
        elif kind == 1:
            typ = [1, 128, 129, 135, 143][k % 5]
            fr = F.v6_frame(58, F.icmp(typ, 0, b"\x00\x01\x00\x02" + pay), tags=tags)
        else:
            doff = int(rng.integers(5, 16))
            bad = rng.random()
            if kind == 3 and bad < 0.3:
                doff = int(rng.integers(0, 5))            # thl < 20
            seg = F.tcp(int(rng.integers(1, 65536)), 80, pay, doff=doff,
                        options=b"\x01" * max(0, doff * 4 - 20))
            if kind == 3 and 0.3 <= bad < 0.6:
                # the data offset past the payload length, the frame long
                # enough to hold it (trailing pad): cl < thl
                seg = F.tcp(int(rng.integers(1, 65536)), 80, pay[:4], doff=15, options=b"")
                pad = b"\x00" * 48
            fr = F.v6_frame(6, seg, tags=tags)
            if kind == 3 and 0.6 <= bad < 0.75:
                # the data offset past the frame itself
                seg = F.tcp(int(rng.integers(1, 65536)), 80, b"", doff=15, options=b"")
                fr = F.v6_frame(6, seg, tags=tags)
        if rng.random() < 0.1:
            b = bytearray(fr)
            b[-1 - int(rng.integers(0, 8))] ^= 0x5A
            fr = bytes(b)
        fr += pad
        if rng.random() < 0.1:
            fr += rng.integers(0, 256, int(rng.integers(1, 9)), dtype=np.uint8).tobytes()
        blobs.append(fr)
    offs, o = [], 0
    for fr in blobs:
        o += 16 * int(rng.integers(0, 3))
        offs.append(o)
        o = (o + len(fr) + 15) & ~15
    umem = np.zeros(offs[-1] + len(blobs[-1]), np.uint8)
    for off, fr in zip(offs, blobs):
        umem[off:off + len(fr)] = np.frombuffer(fr, np.uint8)
    descs = np.zeros(n, xdpgpu.DESC_DTYPE)
    descs["addr"] = offs
    descs["len"] = [len(fr) for fr in blobs]
    return umem, descs


def test_v6_late_frames_cover_aborted_tcp():
    """The generator's TCP cases reach parse_tcphdr's failures (the oracle
    ABORTs them) and the rest of the shapes verify or drop."""
    umem, descs = v6_late_frames(41, 3000)
    v, _, _, st = oracle.process(umem.copy(), descs, 0x5, 0, 2)
    assert (v == xdpgpu.ABORTED).sum() > 50
    assert (v == xdpgpu.REDIRECT).sum() > 1500 and (v == xdpgpu.DROP).sum() > 50
    assert (v == xdpgpu.PASS).sum() > 50          # NDP


@pytest.mark.gpu
@pytest.mark.parametrize("tune,window", SHORT_VARIANTS)
def test_v6_late_frames_vs_oracle(dev, tune, window):
    """Tagged IPv6 and IPv6/TCP through the network_tuple / no-tuple builds
    (late check words and data offsets in the bulk pass) against the
    oracle, with and without the echo responder."""
    umem, descs = v6_late_frames(41, 3000)
    for flags, iv, fmt in ((0x5, 0, 2), (0x4, 7, 0), (0x7, 0x1234, 2), (0x1, 0, 2),
                           (0x7, 0, 1), (0x3, 5, 0)):
        ou = umem.copy()
        ov, ores, otup, ost = oracle.process(ou, descs, flags, iv, fmt)
        v, res, tup, um2, st = run_dev(umem, descs, flags | xdpgpu.CFG_STATS, iv, fmt, window,
                                       tune)
        assert_same((v, res, tup, um2), (ov, ores, otup, ou), f"late/{flags:#x}/fmt{fmt}")
        oracle_stats_match(st, ost)


@pytest.mark.parametrize("tune,window", SHORT_VARIANTS)
def test_v6_build_icmp_vs_oracle(dev, golden, tune, window):
    """The IPv6 builds (network_tuple, no tuple, and any tuple with the echo
    responder): IPv4 ICMP and ICMPv6 other than NDP go through the fast
    shape and the bulk pass, which answers untagged echo requests; the
    golden fixtures, ICMPv6 frames of every type class, the IMIX pool and
    the echo bench leg's pool against the oracle (UMEM after included)."""
    fx, _ = golden
    cases = [("golden", fx["umem"], fx["descs"].view(xdpgpu.DESC_DTYPE)),
             ("icmp6", *icmp6_frames(31, 2000))]
    um, ds, _ = xdpgpu.pool_generate(300000, xdpgpu.POOL_IMIX, 64, 0x5EED0003)
    cases.append(("imix", um, ds))
    um, ds, _ = xdpgpu.pool_generate(200000, xdpgpu.POOL_UDP4, 128, 0x5EED0042,
                                     ppm_echo6=200000)
    cases.append(("echo-pool", um, ds))
    for name, umem, descs in cases:
        # the echo responder with the 16-byte tuple selects the IPv6 build too
        for flags, iv, fmt in ((0x5, 0, 2), (0x4, 7, 0), (0x7, 0x1234, 2), (0x7, 0, 1),
                               (0x6, 3, 0)):
            ou = umem.copy()
            ov, ores, otup, ost = oracle.process(ou, descs, flags, iv, fmt)
            v, res, tup, um2, st = run_dev(umem, descs, flags, iv, fmt, window, tune)
            assert_same((v, res, tup, um2), (ov, ores, otup, ou),
                        f"{name}/{flags:#x}/fmt{fmt}")
            oracle_stats_match(st, ost)
