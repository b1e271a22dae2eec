# SPDX-License-Identifier: GPL-2.0
"""Multi-buffer packets (XDPGPU_CFG_FRAGS): packets of several descriptors,
XDP_PKT_CONTD on all but the last (headers/linux/if_xdp.h:122; IS_EOP_DESC,
xdpsock.c:67; xdpsock's --frags mode, xdpsock.c:1349).

The build processes such a packet as one frame, the concatenation of its
fragments (include/xdpgpu.h).  The reference has no per-packet function
for them (process_packet looks at one descriptor), so the semantics are
build-defined and pinned by equivalence: a pool of frames split into
fragments gives, per packet, exactly the verdict, record, tuple, counters
and echo rewrite of the unsplit frame.

CPU: the oracle against that equivalence, broken packets, the flag off.
GPU: the HIP path (device and host) against the oracle: packets read in
place.
"""
import numpy as np
import pytest

import oracle
import xdpgpu

CONTD = xdpgpu.PKT_CONTD
FRAGS = xdpgpu.CFG_FRAGS


def split_pool(umem, descs, seed, max_frags=4, skew=False):
    """Each frame of (umem, descs) as a packet of 1..max_frags fragments at
    fresh 16-byte aligned offsets (skew: any byte offset); the last fragment
    is followed by the frame's own over-read byte.  Returns the new UMEM,
    the descriptors and the index of each packet's first descriptor."""
    rng = np.random.default_rng(seed)
    pieces, nd, heads, pos = [], [], [], 0
    size = len(umem)
    for d in descs:
        eff = (int(d["addr"]) & ((1 << 48) - 1)) + (int(d["addr"]) >> 48)
        ln = int(d["len"])
        assert eff + ln <= size
        fr = umem[eff:eff + ln].tobytes()
        ob = bytes([int(umem[eff + ln])]) if eff + ln < size else b"\0"
        nf = int(rng.integers(1, max_frags + 1)) if ln > max_frags else 1
        cuts = sorted(rng.choice(np.arange(1, ln), nf - 1, replace=False).tolist()) \
            if nf > 1 else []
        bounds = [0] + cuts + [ln]
        heads.append(len(nd))
        for k in range(nf):
            part = fr[bounds[k]:bounds[k + 1]]
            pos = (pos + 15) & ~15
            if skew:
                pos += int(rng.integers(0, 16))
            pieces.append((pos, part + (ob if k == nf - 1 else b"")))
            nd.append((pos, len(part), CONTD if k < nf - 1 else 0))
            pos += len(part) + 1
    u = np.zeros(pos + 64, np.uint8)
    for p, b in pieces:
        u[p:p + len(b)] = np.frombuffer(b, np.uint8)
    return u, np.array(nd, dtype=xdpgpu.DESC_DTYPE), np.array(heads)


def packet_of(descs):
    """Each descriptor's packet index."""
    contd = (descs["options"] & CONTD) != 0
    starts = np.ones(len(descs), bool)
    starts[1:] = ~contd[:-1]
    return np.cumsum(starts) - 1


def packet_bytes(umem, descs, h):
    """The bytes of the packet whose first descriptor is h."""
    out = b""
    for d in descs[h:]:
        out += umem[int(d["addr"]):int(d["addr"]) + int(d["len"])].tobytes()
        if not int(d["options"]) & CONTD:
            return out
    return out


def frame_bytes(umem, d):
    return umem[int(d["addr"]):int(d["addr"]) + int(d["len"])].tobytes()


_POOLS = {}


def pool(name):
    if name not in _POOLS:
        if name == "imix":
            u, d, _ = xdpgpu.pool_generate(3000, xdpgpu.POOL_IMIX, 64, 0x5EED0003)
        elif name == "udp4_1500":
            u, d, _ = xdpgpu.pool_generate(1000, xdpgpu.POOL_UDP4, 1500, 0x5EED0002)
        else:
            u, d, _ = xdpgpu.pool_generate(3000, xdpgpu.POOL_UDP4, 128, 9, ppm_echo6=200000)
        _POOLS[name] = (u, d)
    return _POOLS[name]


NAMES = ["imix", "udp4_1500", "echo6"]
CFGS = ((0x5, 0, 1), (0x7, 0x9E3779B9, 2))


# ------------------------------------------------------------------ CPU
@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("skew", [False, True])
def test_oracle_packets_equal_frames(name, skew):
    umem, descs = pool(name)
    u2, d2, heads = split_pool(umem, descs, 11, skew=skew)
    assert len(d2) > len(descs)
    pk = packet_of(d2)
    cont = np.setdiff1d(np.arange(len(d2)), heads)
    for flags, iv, fmt in CFGS:
        u1 = umem.copy()
        fv, fres, ftup, fst = oracle.process(u1, descs, flags, iv, fmt)
        u2c = u2.copy()
        pv, pres, ptup, pst = oracle.process(u2c, d2, flags | FRAGS, iv, fmt)
        np.testing.assert_array_equal(pv, fv[pk])
        np.testing.assert_array_equal(pres[heads], fres)
        assert not pres[cont].view(np.uint8).any()
        tb = xdpgpu.TUPLE_BYTES[fmt]
        pt, ft = ptup.reshape(-1, tb), ftup.reshape(-1, tb)
        np.testing.assert_array_equal(pt[heads], ft)
        assert not pt[cont].any()
        assert pst == fst
        for k, h in enumerate(heads):
            if fv[k] == xdpgpu.TX:
                assert packet_bytes(u2c, d2, h) == frame_bytes(u1, descs[k])
    if name == "echo6":
        assert (fv == xdpgpu.TX).sum() > 100


def broken_batches():
    """(umem, descs) with a packet the batch ends inside of, and with a
    fragment outside the UMEM; the first descriptors of those packets."""
    umem, descs = pool("imix")
    u2, d2, heads = split_pool(umem, descs[:300], 5, max_frags=3)
    nfr = np.diff(np.append(heads, len(d2)))
    multi = heads[nfr > 1]
    cut = int(multi[-1])
    bad = d2.copy()
    h2 = int(multi[0])
    bad[h2 + 1]["addr"] = len(u2) + 4096
    return u2, d2[:cut + 1], cut, bad, h2


def test_oracle_broken_packets():
    u2, cutd, cut, bad, h2 = broken_batches()
    # the batch ends inside a packet: ABORTED, counted once with its bytes
    v, res, _, st = oracle.process(u2.copy(), cutd, 0x5 | FRAGS, 0, 1)
    assert v[cut] == xdpgpu.ABORTED and not res[cut:].view(np.uint8).any()
    rv, _, _, rst = oracle.process(u2.copy(), cutd[:cut], 0x5 | FRAGS, 0, 1)
    np.testing.assert_array_equal(v[:cut], rv)
    assert st["frames"] == rst["frames"] + 1
    assert st["bytes"] == rst["bytes"] + int(cutd[cut]["len"])
    assert st["verdict"][xdpgpu.ABORTED] == rst["verdict"][xdpgpu.ABORTED] + 1
    # a fragment outside the UMEM: every descriptor of the packet ABORTED
    v, _, _, _ = oracle.process(u2.copy(), bad, 0x5 | FRAGS, 0, 1)
    k = h2
    while True:
        assert v[k] == xdpgpu.ABORTED
        if not int(bad[k]["options"]) & CONTD:
            break
        k += 1


def test_oracle_flag_off_ignores_options():
    umem, descs = pool("udp4_1500")
    u2, d2, _ = split_pool(umem, descs[:200], 7)
    plain = d2.copy()
    plain["options"] = 0
    a = oracle.process(u2.copy(), d2, 0x5, 0, 1)
    b = oracle.process(u2.copy(), plain, 0x5, 0, 1)
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])
    assert a[3] == b[3] and a[3]["frames"] == len(d2)


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("tune", [0, 512])
@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("skew", [False, True])
def test_gpu_packets_vs_oracle(name, skew, tune):
    from test_gpu_parity import assert_same, oracle_stats_match, run_dev
    umem, descs = pool(name)
    u2, d2, _ = split_pool(umem, descs, 11, skew=skew)
    for flags, iv, fmt in CFGS:
        ou = u2.copy()
        ov, ores, otup, ost = oracle.process(ou, d2, flags | FRAGS, iv, fmt)
        v, res, tup, um, st = run_dev(u2, d2, flags | FRAGS, iv, fmt, 64, tune)
        assert_same((v, res, tup, um), (ov, ores, otup, ou), f"frags/{name}/{flags:#x}")
        oracle_stats_match(st, ost)


@pytest.mark.gpu
def test_gpu_broken_packets():
    from test_gpu_parity import assert_same, oracle_stats_match, run_dev
    u2, cutd, _, bad, _ = broken_batches()
    for descs in (cutd, bad):
        ou = u2.copy()
        ov, ores, otup, ost = oracle.process(ou, descs, 0x5 | FRAGS, 0, 1)
        v, res, tup, um, st = run_dev(u2, descs, 0x5 | FRAGS, 0, 1)
        assert_same((v, res, tup, um), (ov, ores, otup, ou), "frags/broken")
        oracle_stats_match(st, ost)


@pytest.mark.gpu
def test_gpu_host_path_echo():
    """xdpgpu_process on host buffers: echo replies written back into the
    fragments of the registered UMEM."""
    from test_gpu_parity import assert_same
    umem, descs = pool("echo6")
    u2, d2, _ = split_pool(umem, descs, 3)
    ou = u2.copy()
    ov, ores, otup, _ = oracle.process(ou, d2, 0x7 | FRAGS, 0x9E3779B9, 2)
    hu = u2.copy()
    with xdpgpu.XdpGpu(0, 0x7 | FRAGS, 0x9E3779B9, 2) as g:
        g.register_umem(hu)
        v, res, tup = g.process(d2)
    assert_same((v, res, tup.view(np.uint8).reshape(-1), hu), (ov, ores, otup, ou),
                "frags/host")
