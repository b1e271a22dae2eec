# SPDX-License-Identifier: GPL-2.0
"""The host path (xdpgpu_submit / xdpgpu_wait) as an RX loop drives it:
two batches in flight, descriptors of a recycled fill ring (interleaved,
shuffled, reused addresses, a batch that wraps round the ring), ICMPv6 echo
replies written back.  SURVEY §8b ownership: the library writes only the TX
frames' own bytes, so after every batch the whole host UMEM must equal the
oracle run over the same batches in submission order, byte for byte.

The batches two slots hold at once name disjoint frames (an AF_XDP
application cannot hand a frame back to the kernel before its batch is
done: af_xdp_user.c:1087-1106), but their UMEM spans overlap and later
batches receive frames earlier batches rewrote."""
import numpy as np
import pytest

import oracle
import xdpgpu

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

ECHO = 0x7       # verify + echo + stats


def ring_batches(nframes: int, nbatch: int, B: int, seed: int):
    """Frame indices per batch: random frames not in the previous batch
    (recycled, interleaved), one batch that wraps round the end of the
    frame array, and one in strictly cyclic order."""
    rng = np.random.default_rng(seed)
    out = []
    prev = np.zeros(0, np.int64)
    for k in range(nbatch):
        if k == nbatch // 3:
            b = (np.arange(B) + nframes - B // 2) % nframes     # wraps
        elif k == nbatch // 2:
            b = (np.arange(B) * 7 + 3) % nframes                # strided
        else:
            free = np.setdiff1d(np.arange(nframes), prev)
            b = rng.choice(free, B, replace=False)
        if np.intersect1d(b, prev).size:
            free = np.setdiff1d(np.arange(nframes), prev)
            b = rng.choice(free, B, replace=False)
        out.append(b)
        prev = b
    return out


def run_ring(umem, descs, batches, flags, tune, fmt=xdpgpu.TUPLE_NET, pinned=True, window=64,
             chunk=0, host_stats=None):
    """Submit the batches alternately on the two slots, waiting for a slot
    only when it is needed again; returns outputs per batch and stats
    (host_stats, a dict, receives xdpgpu_host_stats)."""
    n_max = max(len(b) for b in batches)
    tb = xdpgpu.TUPLE_BYTES[fmt]
    outs = []
    with xdpgpu.XdpGpu(0, flags, 0x9E3779B9, fmt, window, max_batch=n_max, tune=tune) as ctx:
        ctx.register_umem(umem, chunk)
        bufs = []
        for slot in range(2):
            if pinned:
                d = xdpgpu.HostBuffer(n_max, xdpgpu.DESC_DTYPE)
                v = xdpgpu.HostBuffer(n_max, np.uint8)
                r = xdpgpu.HostBuffer(n_max, xdpgpu.RESULT_DTYPE)
                t = xdpgpu.HostBuffer(n_max * tb, np.uint8)
                bufs.append((d, v, r, t))
            else:
                bufs.append(tuple(type("B", (), {"array": a})() for a in (
                    np.zeros(n_max, xdpgpu.DESC_DTYPE), np.zeros(n_max, np.uint8),
                    np.zeros(n_max, xdpgpu.RESULT_DTYPE), np.zeros(n_max * tb, np.uint8))))
        pending = [None, None]

        def collect(slot):
            k, m = pending[slot]
            ctx.wait(slot)
            d, v, r, t = bufs[slot]
            outs[k] = (v.array[:m].copy(), r.array[:m].copy(), t.array[: m * tb].copy())
            pending[slot] = None

        for k, b in enumerate(batches):
            slot = k & 1
            if pending[slot] is not None:
                collect(slot)
            outs.append(None)
            d, v, r, t = bufs[slot]
            m = len(b)
            d.array[:m] = descs[b]
            ctx.submit(slot, d.array[:m], v.array[:m], r.array[:m], t.array[: m * tb])
            pending[slot] = (k, m)
        for slot in range(2):
            if pending[slot] is not None:
                collect(slot)
        st = ctx.stats()
        if host_stats is not None:
            host_stats.update(ctx.host_stats())
        for bb in bufs:
            for x in bb:
                if hasattr(x, "close"):
                    x.close()
    return outs, st


def oracle_ring(umem, descs, batches, flags, fmt=xdpgpu.TUPLE_NET):
    outs = []
    tot = None
    for b in batches:
        v, res, tup, st = oracle.process(umem, np.ascontiguousarray(descs[b]), flags,
                                         0x9E3779B9, fmt)
        outs.append((v, res.view(np.uint8).reshape(-1), tup))
        if tot is None:
            tot = st
        else:
            for key in ("frames", "bytes", "l3_bad", "l4_bad", "l4_absent", "frag"):
                tot[key] += st[key]
            tot["verdict"] = [a + c for a, c in zip(tot["verdict"], st["verdict"])]
    return outs, tot


@pytest.mark.parametrize("tune", [0], ids=["span_copy"])
@pytest.mark.parametrize("pinned", [True, False], ids=["pinned", "pageable"])
@pytest.mark.parametrize("window", [64, 0], ids=["w64", "wauto"])
def test_ring_echo_two_slots(tune, pinned, window):
    nframes = 16384
    umem, descs, _ = xdpgpu.pool_generate(nframes, xdpgpu.POOL_UDP4, 128, 31,
                                          ppm_echo6=300000)
    batches = ring_batches(nframes, 24, 2048, 5)
    host = umem.copy()
    got, st = run_ring(host, descs, batches, ECHO, tune, pinned=pinned, window=window)
    ou = umem.copy()
    want, ost = oracle_ring(ou, descs, batches, ECHO)
    ntx = 0
    for k, (g, w) in enumerate(zip(got, want)):
        np.testing.assert_array_equal(g[0], w[0], err_msg=f"batch {k} verdicts")
        np.testing.assert_array_equal(g[1].view(np.uint8).reshape(-1), w[1],
                                      err_msg=f"batch {k} results")
        np.testing.assert_array_equal(g[2], w[2], err_msg=f"batch {k} tuples")
        ntx += int((w[0] == xdpgpu.TX).sum())
    assert ntx > 1000, "the pool must exercise the echo responder"
    # replies that came round again are REDIRECTed (type 129 is no request)
    assert np.array_equal(host, ou), "host UMEM differs from the oracle's"
    assert st["frames"] == ost["frames"]
    assert [st["verdict"][x] for x in xdpgpu.VERDICT_NAMES] == ost["verdict"]


def test_tx_only_write_back():
    """Bytes of frames outside the batch, and of non-TX frames, are never
    written: the host changes them while the batch is in flight (as a NIC
    refilling fill-ring frames would) and the changes survive."""
    nframes = 4096
    umem, descs, _ = xdpgpu.pool_generate(nframes, xdpgpu.POOL_UDP4, 128, 32,
                                          ppm_echo6=500000)
    host = umem.copy()
    batch = np.arange(0, nframes, 2)                 # every other frame
    with xdpgpu.XdpGpu(0, ECHO, 0, xdpgpu.TUPLE_V4, max_batch=len(batch)) as ctx:
        ctx.register_umem(host)
        d = np.ascontiguousarray(descs[batch])
        v = np.zeros(len(batch), np.uint8)
        ctx.submit(0, d, v)
        # the odd frames are not in the batch: scribble on them now
        for f in range(1, nframes, 2):
            a = int(descs["addr"][f])
            host[a:a + 64] = 0xA5
        ctx.wait(0)
    ou = umem.copy()
    ov, _, _, _ = oracle.process(ou, d, ECHO, 0, 1)
    np.testing.assert_array_equal(v, ov)
    for f in range(1, nframes, 2):
        a = int(descs["addr"][f])
        ou[a:a + 64] = 0xA5
    assert np.array_equal(host, ou)


@pytest.mark.parametrize("mode", ["copies", "gather", "compact"])
def test_frags_ring_host_path(mode):
    """Multi-buffer packets on the host path, two slots in flight, echo on:
    every fragment's bytes only as the oracle writes them.  With the gather
    (the UMEM registered with a chunk size) or the host compaction every
    fragment takes the byte after it, so the packet's over-read byte after
    its last fragment is there."""
    gather = mode == "gather"
    flags = {"copies": 0, "gather": xdpgpu.CFG_UMEM_GATHER,
             "compact": xdpgpu.CFG_HOST_COMPACT}[mode]
    import test_frags as TF
    umem, descs = TF.pool("echo6")
    u2, d2, _ = TF.split_pool(umem, descs, 3)
    # packets = runs of descriptors; batches of whole packets
    heads = np.nonzero(np.r_[True, (d2["options"][:-1] & xdpgpu.PKT_CONTD) == 0])[0]
    bounds = np.r_[heads, len(d2)]
    per = 64
    batches = []
    for p0 in range(0, len(heads), per):
        batches.append(np.arange(bounds[p0], bounds[min(p0 + per, len(heads))]))
    host = u2.copy()
    hs = {}
    got, st = run_ring(host, d2, batches, ECHO | xdpgpu.CFG_FRAGS | flags, 0,
                       fmt=xdpgpu.TUPLE_V4, chunk=4096 if mode != "copies" else 0,
                       host_stats=hs)
    assert hs["umem_gathers"] == (len(batches) if gather else 0), hs
    assert hs["umem_compacted"] == (len(batches) if mode == "compact" else 0), hs
    ou = u2.copy()
    want, ost = oracle_ring(ou, d2, batches, ECHO | xdpgpu.CFG_FRAGS, fmt=xdpgpu.TUPLE_V4)
    for k, (g, w) in enumerate(zip(got, want)):
        np.testing.assert_array_equal(g[0], w[0], err_msg=f"batch {k} verdicts")
    assert np.array_equal(host, ou)
    assert st["frames"] == ost["frames"]


def test_process_dev_two_streams():
    """Launches of one context on two streams share its scratch (deferral
    lists, counts): the context orders them, and each batch's outputs
    equal the oracle's.  IMIX defers many frames, so an unordered pair of
    launches would mix the lists."""
    from test_gpu_parity import to_dev
    pools = [xdpgpu.pool_generate(200000, xdpgpu.POOL_IMIX, 64, s) for s in (41, 42)]
    want = [oracle.process(u.copy(), d, 0x5, 0, 2)[:3] for u, d, _ in pools]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    with xdpgpu.XdpGpu(0, 0x5, 0, xdpgpu.TUPLE_NET) as ctx:
        bufs = []
        for u, d, _ in pools:
            n = len(d)
            bufs.append((to_dev(u), u.nbytes, to_dev(d, 16), n,
                         torch.empty(n, dtype=torch.uint8, device="cuda:0"),
                         torch.empty(n * 16, dtype=torch.uint8, device="cuda:0"),
                         torch.empty(n * 44, dtype=torch.uint8, device="cuda:0")))
        torch.cuda.synchronize()
        for rep in range(6):
            k = rep & 1
            du, us, dd, n, dv, dr, dt = bufs[k]
            ctx.process_dev(du, us, dd, n, dv, dr, dt, stream=streams[k])
        torch.cuda.synchronize()
        for k in range(2):
            du, us, dd, n, dv, dr, dt = bufs[k]
            wv, wres, wtup = want[k]
            np.testing.assert_array_equal(dv.cpu().numpy(), wv)
            np.testing.assert_array_equal(dr.cpu().numpy(), wres.view(np.uint8).reshape(-1))
            np.testing.assert_array_equal(dt.cpu().numpy(), wtup)


def test_queue_stats():
    """Per-queue counters (af_xdp_kern.c:19-24, :157-160): contexts of one
    RX queue add up, a closed context's counters are kept, other queues
    are apart."""
    from test_gpu_parity import to_dev
    qa, qb = 1000 + np.random.randint(1 << 20), 2000 + np.random.randint(1 << 20)
    pools = [xdpgpu.pool_generate(n, xdpgpu.POOL_IMIX, 64, s) for n, s in ((30000, 51),
                                                                           (20000, 52))]
    want = [oracle.process(u.copy(), d, 0x5, 0, 1)[3] for u, d, _ in pools]
    ctxs = [xdpgpu.XdpGpu(0, 0x5, 0, 1, queue_id=q) for q in (qa, qa, qb)]
    keep = []      # the device buffers live until the launches are done
    for c, (u, d, _) in zip(ctxs, (pools[0], pools[1], pools[0])):
        n = len(d)
        bufs = (to_dev(u), to_dev(d, 16), torch.empty(n, dtype=torch.uint8, device="cuda:0"),
                torch.empty(n * 16, dtype=torch.uint8, device="cuda:0"),
                torch.empty(n * 16, dtype=torch.uint8, device="cuda:0"))
        keep.append(bufs)
        c.process_dev(bufs[0], u.nbytes, bufs[1], n, *bufs[2:])
    torch.cuda.synchronize()
    a = xdpgpu.queue_stats(qa)
    assert a["frames"] == want[0]["frames"] + want[1]["frames"]
    assert [a["verdict"][x] for x in xdpgpu.VERDICT_NAMES] == \
        [p + q for p, q in zip(want[0]["verdict"], want[1]["verdict"])]
    b = xdpgpu.queue_stats(qb)
    assert b["frames"] == want[0]["frames"] and b["bytes"] == want[0]["bytes"]
    ctxs[1].close()
    assert xdpgpu.queue_stats(qa)["frames"] == a["frames"]      # kept after close
    for c in ctxs:
        c.close()
    assert xdpgpu.queue_stats(qa) == a
    assert xdpgpu.queue_stats(qb) == b


def test_process_dev_own_and_caller_streams():
    """Launches alternating between the context's own stream (stream None:
    the scratch event is recorded only when another stream comes) and two
    caller streams: every batch's outputs equal the oracle's."""
    from test_gpu_parity import to_dev
    pools = [xdpgpu.pool_generate(150000, xdpgpu.POOL_IMIX, 64, s) for s in (43, 44, 45)]
    want = [oracle.process(u.copy(), d, 0x5, 0, 2)[:3] for u, d, _ in pools]
    streams = [None, torch.cuda.Stream(), None, torch.cuda.Stream(), None]
    with xdpgpu.XdpGpu(0, 0x5, 0, xdpgpu.TUPLE_NET) as ctx:
        bufs = []
        for u, d, _ in pools:
            n = len(d)
            bufs.append((to_dev(u), u.nbytes, to_dev(d, 16), n,
                         torch.empty(n, dtype=torch.uint8, device="cuda:0"),
                         torch.empty(n * 16, dtype=torch.uint8, device="cuda:0"),
                         torch.empty(n * 44, dtype=torch.uint8, device="cuda:0")))
        torch.cuda.synchronize()
        for rep in range(10):
            k = rep % 3
            du, us, dd, n, dv, dr, dt = bufs[k]
            ctx.process_dev(du, us, dd, n, dv, dr, dt, stream=streams[rep % len(streams)])
        torch.cuda.synchronize()
        for k in range(3):
            du, us, dd, n, dv, dr, dt = bufs[k]
            wv, wres, wtup = want[k]
            np.testing.assert_array_equal(dv.cpu().numpy(), wv)
            np.testing.assert_array_equal(dr.cpu().numpy(), wres.view(np.uint8).reshape(-1))
            np.testing.assert_array_equal(dt.cpu().numpy(), wtup)


def test_device_entry_points_reject_host_memory():
    """No kernel of the library dereferences host memory:
    a *_dev call whose UMEM is pinned host memory (mapped into the GPU at
    its own address) or plain pageable memory fails with -EINVAL before
    any launch, and the context stays usable."""
    from test_gpu_parity import to_dev
    umem, descs, expect = xdpgpu.pool_generate(4096, xdpgpu.POOL_UDP4, 64, 61)
    n = len(descs)
    dd = to_dev(descs, 16)
    dv = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    pinned = xdpgpu.HostBuffer(umem.nbytes + 64, np.uint8)
    pinned.array[: umem.nbytes] = umem
    with xdpgpu.XdpGpu(0, 0x5, 0, 1) as ctx:
        for host in (pinned.array, umem):
            with pytest.raises(xdpgpu.XdpGpuError, match="-22|Invalid"):
                ctx.process_dev(host, umem.nbytes, dd, n, dv)
            # the two-slot form checks the same way, on either slot
            for slot in (0, 1):
                with pytest.raises(xdpgpu.XdpGpuError, match="-22|Invalid"):
                    ctx.submit_dev(slot, host, umem.nbytes, dd, n, dv)
        du = to_dev(umem)
        ctx.process_dev(du, umem.nbytes, dd, n, dv)
        torch.cuda.synchronize()
    pinned.close()
    np.testing.assert_array_equal(dv.cpu().numpy(), expect)


@pytest.mark.parametrize("window", [64, 0], ids=["w64", "wauto"])
def test_scattered_batch_runs(window):
    """A batch scattered over a large UMEM (a recycled fill ring's order)
    is copied as at most 64 merged runs, never by reading the host UMEM
    from a kernel: every frame's outputs equal the oracle's, and frames
    outside the batch are never written back."""
    nframes = 1 << 16
    umem, descs, _ = xdpgpu.pool_generate(nframes, xdpgpu.POOL_UDP4, 128, 62,
                                          ppm_echo6=300000)
    rng = np.random.default_rng(63)
    batch = np.sort(rng.choice(nframes, 3000, replace=False))[::-1].copy()
    host = umem.copy()
    d = np.ascontiguousarray(descs[batch])
    with xdpgpu.XdpGpu(0, ECHO, 0, xdpgpu.TUPLE_V4, window, max_batch=len(batch)) as ctx:
        ctx.register_umem(host)
        v, res, tup = ctx.process(d)
    ou = umem.copy()
    ov, ores, otup, _ = oracle.process(ou, d, ECHO, 0, 1)
    np.testing.assert_array_equal(v, ov)
    np.testing.assert_array_equal(res.view(np.uint8).reshape(-1), ores.view(np.uint8).reshape(-1))
    assert int((ov == xdpgpu.TX).sum()) > 100
    assert np.array_equal(host, ou)


CHUNK, HEADROOM = 4096, 256     # af_xdp_user.c:56-57; XDP_PACKET_HEADROOM


def chunked_pool(n, kind, size, seed, **kw):
    return xdpgpu.pool_generate(n, kind, size, seed, stride=CHUNK, headroom=HEADROOM, **kw)


def check_ring(got, want, host, ou, st, ost):
    for k, (g, w) in enumerate(zip(got, want)):
        np.testing.assert_array_equal(g[0], w[0], err_msg=f"batch {k} verdicts")
        np.testing.assert_array_equal(g[1].view(np.uint8).reshape(-1), w[1],
                                      err_msg=f"batch {k} results")
        np.testing.assert_array_equal(g[2], w[2], err_msg=f"batch {k} tuples")
    assert np.array_equal(host, ou), "host UMEM differs from the oracle's"
    assert st["frames"] == ost["frames"]
    assert [st["verdict"][x] for x in xdpgpu.VERDICT_NAMES] == ost["verdict"]


def gather_bytes(descs, batches, usize, over_all=False, packed=False):
    """The 16-byte pieces umem_gather_kernel reads for the batches; packed:
    the bytes XDPGPU_CFG_HOST_COMPACT's staging holds (each piece padded
    to 16 bytes)."""
    tot = 0
    for b in batches:
        raw = descs["addr"][b].astype(np.uint64)
        a = ((raw & np.uint64((1 << 48) - 1)) + (raw >> np.uint64(48))).astype(np.int64)
        ln = descs["len"][b].astype(np.int64)
        ok = (a < usize) & (ln <= usize - a)
        hi = np.minimum(a + ln + (1 if over_all else (ln & 1)), usize)
        piece = np.minimum((hi + 15) & ~15, usize) - (a & ~15)
        if packed:
            piece = (piece + 15) & ~15
        tot += int(piece[ok].sum())
    return tot


# how a chunked UMEM's frames reach the device: the copy engine's rows,
# the gather kernel, or the host threads' compaction
MODE_FLAGS = {"rows": 0, "gather": xdpgpu.CFG_UMEM_GATHER, "compact": xdpgpu.CFG_HOST_COMPACT}


@pytest.mark.parametrize("mode,pinned", [("rows", True), ("gather", True), ("gather", False),
                                         ("compact", True), ("compact", False)],
                         ids=["rows", "gather", "gather_pageable_descs", "compact",
                              "compact_pageable_descs"])
@pytest.mark.parametrize("kind,size,ppm", [(xdpgpu.POOL_UDP4, 64, 300000),
                                           (xdpgpu.POOL_IMIX, 64, 200000)],
                         ids=["udp64", "imix"])
def test_ring_chunked_umem(kind, size, ppm, mode, pinned):
    """The reference's UMEM geometry (4 KiB chunks, each frame at its
    chunk's headroom) registered with its chunk size: the host path copies
    one window of each chunk (rows of a pitched copy), or with
    XDPGPU_CFG_UMEM_GATHER a kernel gathers each frame's bytes (reading
    page-locked descriptor arrays through their GPU mapping, pageable ones
    after their copy), or with XDPGPU_CFG_HOST_COMPACT the host threads
    pack the same bytes into one transfer.  Recycled,
    wrapping and strided batches (the scattered path merges chunk runs),
    echo replies written back: outputs and the whole host UMEM equal the
    oracle's."""
    nframes = 8192
    umem, descs, _ = chunked_pool(nframes, kind, size, 71, ppm_echo6=ppm)
    assert int(descs["addr"][1]) == CHUNK + HEADROOM
    batches = ring_batches(nframes, 12, 1024, 72)
    host = umem.copy()
    hs = {}
    flags = ECHO | MODE_FLAGS[mode]
    got, st = run_ring(host, descs, batches, flags, 0, window=0, chunk=CHUNK, host_stats=hs,
                       pinned=pinned)
    ou = umem.copy()
    want, ost = oracle_ring(ou, descs, batches, ECHO)
    check_ring(got, want, host, ou, st, ost)
    ntx = sum(int((w[0] == xdpgpu.TX).sum()) for w in want)
    assert ntx > 100
    assert hs["frames"] == sum(len(b) for b in batches)
    if mode == "gather":
        assert hs["umem_gathers"] == len(batches), hs
        assert hs["umem_h2d_bytes"] == gather_bytes(descs, batches, umem.size), hs
        return
    if mode == "compact":
        assert hs["umem_compacted"] == hs["umem_copies"] == len(batches), hs
        assert hs["umem_gathers"] == 0, hs
        assert hs["umem_h2d_bytes"] == gather_bytes(descs, batches, umem.size,
                                                    packed=True), hs
        return
    assert hs["umem_gathers"] == 0, hs
    # at most one window of every chunk per batch (random recycled batches
    # merge their chunk runs, copying the rows between), always below the
    # span copy's whole chunks
    lens = descs["len"].astype(np.int64)
    width = int(lens.max()) + 1
    assert hs["umem_h2d_bytes"] <= len(batches) * nframes * width, hs
    assert hs["umem_h2d_bytes"] < len(batches) * nframes * CHUNK // 2, hs


@pytest.mark.parametrize("mode", ["rows", "gather", "compact"])
def test_chunked_consecutive_bytes(mode):
    """Consecutive 64 B frames in 4 KiB chunks: exactly one row of the
    batch's window (its longest frame and udp_csum's over-read byte) per
    chunk, one copy per batch, or (gather) each frame's own 64 bytes;
    outputs equal the oracle's."""
    nframes, B = 4096, 1024
    umem, descs, _ = chunked_pool(nframes, xdpgpu.POOL_UDP4, 64, 73)
    batches = [np.arange(k, k + B) for k in range(0, nframes, B)]
    host = umem.copy()
    hs = {}
    flags = 0x5 | MODE_FLAGS[mode]
    got, st = run_ring(host, descs, batches, flags, 0, fmt=xdpgpu.TUPLE_V4, window=0,
                       chunk=CHUNK, host_stats=hs)
    ou = umem.copy()
    want, ost = oracle_ring(ou, descs, batches, 0x5, fmt=xdpgpu.TUPLE_V4)
    check_ring(got, want, host, ou, st, ost)
    if mode == "compact":
        # the descriptors and one 4-byte piece offset a frame; each frame's
        # 64 bytes at the chunk's headroom (+ the over-read byte only for
        # odd lengths): 64 bytes in one transfer a batch
        assert hs["desc_h2d_bytes"] == nframes * (16 + 4), hs
        assert hs["umem_h2d_bytes"] == gather_bytes(descs, batches, umem.size, packed=True)
        assert hs["umem_compacted"] == hs["umem_copies"] == len(batches), hs
        return
    assert hs["desc_h2d_bytes"] == nframes * 16
    if mode == "gather":
        assert hs["umem_h2d_bytes"] == gather_bytes(descs, batches, umem.size), hs
        assert hs["umem_h2d_bytes"] <= nframes * 64, hs
        assert hs["umem_gathers"] == hs["umem_copies"] == len(batches), hs
        return
    lens = descs["len"].astype(np.int64)
    # every frame sits at the chunk's headroom: a batch's window is its
    # longest frame + 1, once per chunk
    assert hs["umem_h2d_bytes"] == sum(len(b) * (int(lens[b].max()) + 1) for b in batches), hs
    assert hs["umem_copies"] == len(batches), hs


def test_compact_thread_counts():
    """XDPGPU_CFG_HOST_COMPACT with 1, 3 and 7 packing threads (uneven shares
    of an odd batch, IMIX frames with tags and IPv6 in 4 KiB chunks) and the
    default count: outputs equal the oracle's every time, the same bytes
    move, and the count cannot change while a slot is in flight."""
    nframes = 3001
    umem, descs, _ = chunked_pool(nframes, xdpgpu.POOL_IMIX, 64, 79)
    ov, ores, otup, _ = oracle.process(umem.copy(), descs, 0x5, 0, xdpgpu.TUPLE_V4)
    flags = 0x5 | xdpgpu.CFG_HOST_COMPACT
    with xdpgpu.XdpGpu(0, flags, 0, xdpgpu.TUPLE_V4, 0, max_batch=nframes) as ctx:
        ctx.register_umem(umem, CHUNK)
        assert 1 <= ctx.host_threads(0) <= 16
        for t in (1, 3, 7, 0):
            got = ctx.host_threads(t)
            assert got == t or t == 0
            h0 = ctx.host_stats()
            v, r, tup = ctx.process(descs)
            h1 = ctx.host_stats()
            np.testing.assert_array_equal(v, ov, err_msg=f"{t} threads")
            assert r.tobytes() == ores.tobytes() and tup.tobytes() == otup.tobytes()
            assert h1["umem_compacted"] - h0["umem_compacted"] == 1
            assert (h1["umem_h2d_bytes"] - h0["umem_h2d_bytes"] ==
                    gather_bytes(descs, [np.arange(nframes)], umem.size, packed=True))
        hv = np.zeros(nframes, np.uint8)
        ctx.submit(0, descs, hv)
        with pytest.raises(xdpgpu.XdpGpuError, match="EBUSY|busy|in flight"):
            ctx.host_threads(2)
        ctx.wait(0)
        np.testing.assert_array_equal(hv, ov)


def udp_to_frame_end(umem, descs, length):
    """Frames of `length` bytes whose IPv4 and UDP lengths run to the
    frame's last byte (the pools pad odd sizes), the IPv4 header checksum
    redone: a UDP checksum range of odd length then ends at the frame's
    end, and udp_csum reads the byte after it."""
    for a in descs["addr"][descs["len"] >= length].astype(np.int64):
        f = umem[a:a + length]
        if f[12] != 0x08 or f[13] != 0x00 or f[23] != 17:
            continue
        f[16:18] = np.frombuffer((length - 14).to_bytes(2, "big"), np.uint8)
        f[38:40] = np.frombuffer((length - 34).to_bytes(2, "big"), np.uint8)
        f[24:26] = 0
        w = f[14:34].astype(np.uint32)
        c = int((w[0::2] << 8).sum() + w[1::2].sum())
        while c >> 16:
            c = (c & 0xffff) + (c >> 16)
        f[24:26] = np.frombuffer((~c & 0xffff).to_bytes(2, "big"), np.uint8)
    descs["len"][descs["len"] >= length] = length


def test_two_queues_share_a_umem():
    """Two contexts (two RX queues) register the same UMEM, as the
    reference's sockets share one; both run batches, one closes first, the
    other still runs, and a context made afterwards runs too: a failed
    second unregistration must not surface as the next launch's error."""
    nframes = 4096
    umem, descs, _ = xdpgpu.pool_generate(nframes, xdpgpu.POOL_UDP4, 64, 77)
    want, _, _, _ = oracle.process(umem.copy(), descs, 0x5, 0, xdpgpu.TUPLE_V4)

    def batch(ctx, lo, hi):
        v, _, _ = ctx.process(descs[lo:hi], want_res=False, want_tup=False)
        np.testing.assert_array_equal(v, want[lo:hi])

    a = xdpgpu.XdpGpu(0, 0x5, 0, xdpgpu.TUPLE_V4, 0)
    b = xdpgpu.XdpGpu(0, 0x5, 0, xdpgpu.TUPLE_V4, 0)
    try:
        a.register_umem(umem)
        b.register_umem(umem)
        batch(a, 0, 2048)
        batch(b, 2048, 4096)
        a.close()
        batch(b, 0, 4096)
        b.close()
        with xdpgpu.XdpGpu(0, 0x5, 0, xdpgpu.TUPLE_V4, 0) as c:
            c.register_umem(umem.copy())
            batch(c, 0, 4096)
    finally:
        a.close()
        b.close()


def test_two_queues_share_a_umem_gather():
    """The gather form of the shared UMEM (XDPGPU_CFG_UMEM_GATHER reads the
    registered UMEM through its GPU mapping): both contexts hold the one
    registration (xdpgpu_host_pin_refs counts them), queue A closes and
    queue B's next gathered batch still reads mapped memory, bit-exact; the
    last close releases the pinning."""
    nframes, B = 4096, 2048
    umem, descs, _ = chunked_pool(nframes, xdpgpu.POOL_UDP4, 64, 78)
    want, wres, _, _ = oracle.process(umem.copy(), descs, 0x5, 0, xdpgpu.TUPLE_V4)
    flags = 0x5 | xdpgpu.CFG_UMEM_GATHER

    def batch(ctx, lo, hi):
        v, r, _ = ctx.process(descs[lo:hi], want_res=True, want_tup=False)
        np.testing.assert_array_equal(v, want[lo:hi])
        np.testing.assert_array_equal(r.view(np.uint8).reshape(-1),
                                      wres[lo:hi].view(np.uint8).reshape(-1))

    assert xdpgpu.host_pin_refs(umem) == 0
    a = xdpgpu.XdpGpu(0, flags, 0, xdpgpu.TUPLE_V4, 0, max_batch=nframes)
    b = xdpgpu.XdpGpu(0, flags, 0, xdpgpu.TUPLE_V4, 0, max_batch=nframes)
    try:
        a.register_umem(umem, CHUNK)
        b.register_umem(umem, CHUNK)
        assert xdpgpu.host_pin_refs(umem) == 2
        g0 = b.host_stats()["umem_gathers"]
        batch(a, 0, B)
        batch(b, B, nframes)
        a.close()
        assert xdpgpu.host_pin_refs(umem) == 1
        batch(b, 0, nframes)
        assert b.host_stats()["umem_gathers"] == g0 + 2
        b.close()
        assert xdpgpu.host_pin_refs(umem) == 0
    finally:
        a.close()
        b.close()


def test_gather_descs_inside_pinned_buffer():
    """The gather reads page-locked descriptors through their GPU mapping:
    a batch handed over as a slice from the middle of a page-locked array
    (an RX loop's descriptor ring) is read at its own offset."""
    nframes, B = 4096, 1000
    umem, descs, _ = chunked_pool(nframes, xdpgpu.POOL_UDP4, 64, 76)
    ring = xdpgpu.HostBuffer(3 * B, xdpgpu.DESC_DTYPE)
    outs = [xdpgpu.HostBuffer(B, dt) for dt in (np.uint8, xdpgpu.RESULT_DTYPE,
                                                  xdpgpu.TUPLE4_DTYPE)]
    try:
        with xdpgpu.XdpGpu(0, 0x5 | xdpgpu.CFG_UMEM_GATHER, 0, xdpgpu.TUPLE_V4, 0,
                           max_batch=B) as ctx:
            ctx.register_umem(umem, CHUNK)
            for k, lo in enumerate((B + 13, 7, 2 * B - 1)):
                b = np.arange(k * B, (k + 1) * B) % nframes
                ring.array[lo:lo + B] = descs[b]
                v, r, t = (o.array for o in outs)
                ctx.submit(0, ring.array[lo:lo + B], v, r, t)
                ctx.wait(0)
                ov, ores, otup, _ = oracle.process(umem.copy(), np.ascontiguousarray(descs[b]),
                                                   0x5, 0, xdpgpu.TUPLE_V4)
                np.testing.assert_array_equal(v, ov, err_msg=f"batch at {lo}")
                np.testing.assert_array_equal(r.view(np.uint8).reshape(-1),
                                              ores.view(np.uint8).reshape(-1))
            assert ctx.host_stats()["umem_gathers"] == 3
    finally:
        ring.close()
        for o in outs:
            o.close()


@pytest.mark.parametrize("mode", ["gather", "compact"])
@pytest.mark.parametrize("size", [64, 65, 67, 600, 601])
def test_gather_over_read_byte(size, mode):
    """The gather copies a frame's own bytes and, for odd lengths, the byte
    after it (udp_csum's over-read, lib_checksum.h:175-176): frames whose
    UDP range runs to their last byte, every other byte of the 4 KiB chunks
    random, so a byte the kernels read but the gather left out would show
    as the mirror's stale value.  Outputs equal the oracle's on the host
    UMEM; for odd sizes the over-read byte is shown to matter (changing it
    changes the oracle's records)."""
    nframes, B = 2048, 512
    umem, descs, _ = chunked_pool(nframes, xdpgpu.POOL_UDP4, size + (size & 1), 75)
    udp_to_frame_end(umem, descs, size)
    lens = descs["len"].astype(np.int64)
    addr = descs["addr"].astype(np.int64)
    assert (lens == size).mean() > 0.9
    inr = addr + lens <= umem.size
    keep = np.zeros(umem.size + 1, np.int64)
    np.add.at(keep, addr[inr], 1)
    np.add.at(keep, (addr + lens)[inr], -1)
    noise = ~np.cumsum(keep)[:-1].astype(bool)
    umem[noise] = np.random.default_rng(size).integers(0, 256, int(noise.sum()), np.uint8)
    batches = [np.arange(k, k + B) for k in range(0, nframes, B)]
    host = umem.copy()
    hs = {}
    got, st = run_ring(host, descs, batches, 0x4 | MODE_FLAGS[mode], 0,
                       fmt=xdpgpu.TUPLE_V4, window=0, chunk=CHUNK, host_stats=hs)
    ou = umem.copy()
    want, ost = oracle_ring(ou, descs, batches, 0x4, fmt=xdpgpu.TUPLE_V4)
    check_ring(got, want, host, ou, st, ost)
    packed = mode == "compact"
    assert hs["umem_gathers" if not packed else "umem_compacted"] == len(batches), hs
    assert hs["umem_h2d_bytes"] == gather_bytes(descs, batches, umem.size, packed=packed), hs
    assert ost["verdict"][xdpgpu.REDIRECT] > 0.9 * nframes
    z = umem.copy()
    idx = (addr + lens)[inr & (addr + lens < umem.size)]
    z[idx] = umem[idx] + 1
    w2, _ = oracle_ring(z, descs, batches, 0x4, fmt=xdpgpu.TUPLE_V4)
    assert (size & 1) == any(not np.array_equal(a[1], b[1]) for a, b in zip(want, w2))


@pytest.mark.parametrize("mode", ["rows", "gather", "compact"])
def test_chunked_fallbacks_and_umem_end(mode):
    """The rows' edges: a frame whose over-read byte lies in the next chunk
    (the batch falls back to span copies; the gather reads the byte from
    the next chunk), and a UMEM whose size is not a whole number of chunks,
    its last frame cut by the UMEM's end (the last row is copied clamped,
    never read past the host UMEM; the gather skips the frame the UMEM does
    not hold)."""
    nframes = 600
    umem, descs, _ = chunked_pool(nframes, xdpgpu.POOL_UDP4, 64, 74)
    # frame 5 fills its chunk to the last byte: udp_csum reads one past it
    d = descs.copy()
    d["addr"][5] = 5 * CHUNK + HEADROOM
    d["len"][5] = CHUNK - HEADROOM
    cut = (nframes - 1) * CHUNK + HEADROOM + 40          # the last frame cut at 40 bytes
    small = np.ascontiguousarray(umem[:cut])
    for name, u, batch in (("over-read into the next chunk", umem, np.arange(0, 64)),
                           ("UMEM end", small, np.arange(nframes - 300, nframes))):
        host = u.copy()
        hs = {}
        got, st = run_ring(host, d, [batch], 0x5 | MODE_FLAGS[mode],
                           0, fmt=xdpgpu.TUPLE_V4, window=0, chunk=CHUNK, host_stats=hs)
        ou = u.copy()
        want, ost = oracle_ring(ou, d, [batch], 0x5, fmt=xdpgpu.TUPLE_V4)
        check_ring(got, want, host, ou, st, ost)
        assert hs["frames"] == len(batch), name
        assert hs["umem_gathers"] == (1 if mode == "gather" else 0), (name, hs)
        assert hs["umem_compacted"] == (1 if mode == "compact" else 0), (name, hs)
        if mode != "rows":
            assert hs["umem_h2d_bytes"] == gather_bytes(d, [batch], u.size,
                                                        packed=mode == "compact"), (name, hs)
