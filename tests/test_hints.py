# SPDX-License-Identifier: GPL-2.0
"""XDP hints in front of each frame (xdpgpu_hints_dev): the metadata structs
of AF_XDP-interaction/af_xdp_kern.c:42-105 (xdp_hints_rx_time, 16 bytes;
xdp_hints_mark, 8 bytes; the BTF id last, right before the frame) read as
print_meta_info_via_btf does (af_xdp_user.c:813-829).

CPU: the oracle against the structs written here with struct.pack, frame
by frame (the layout of af_xdp_kern.c: packed, BTF id last).  GPU: the HIP
kernel against the oracle."""
import struct

import numpy as np
import pytest

import oracle
import xdpgpu

RX_TIME, MARK = 0x1234, 0x77


def hinted_pool(seed, n=5000, stride=256):
    """Frames at random offsets (any alignment) with rx_time, mark, unknown
    or no metadata in front; returns umem, descs and the expected records."""
    rng = np.random.default_rng(seed)
    umem = np.zeros(n * stride + 64, np.uint8)
    descs = np.zeros(n, xdpgpu.DESC_DTYPE)
    want = np.zeros(n, xdpgpu.HINTS_DTYPE)
    for k in range(n):
        base = k * stride
        head = int(rng.integers(0, 40)) if k else int(rng.integers(0, 20))
        eff = base + head
        descs[k] = (eff, 64, 0)
        kind = int(rng.integers(0, 5))
        ktime, val = int(rng.integers(0, 1 << 63)), int(rng.integers(0, 1 << 32))
        if kind == 0 and eff >= 16:           # struct xdp_hints_rx_time
            umem[eff - 16:eff] = np.frombuffer(struct.pack("<QII", ktime, val, RX_TIME),
                                               np.uint8)
            want[k] = (ktime, val, RX_TIME)
        elif kind == 1 and eff >= 8:          # struct xdp_hints_mark
            umem[eff - 8:eff] = np.frombuffer(struct.pack("<II", val, MARK), np.uint8)
            want[k] = (0, val, MARK)
        elif kind == 2 and eff >= 4:          # an id the application does not know
            umem[eff - 4:eff] = np.frombuffer(struct.pack("<I", 0x999), np.uint8)
            want[k] = (0, 0, 0x999)
        # kind 3, 4: no metadata (id 0)
    return umem, descs, want


def test_oracle_hints():
    umem, descs, want = hinted_pool(1)
    got = oracle.hints(umem, descs, RX_TIME, MARK)
    np.testing.assert_array_equal(got, want)
    assert (want["btf_id"] == RX_TIME).sum() > 500 and (want["btf_id"] == MARK).sum() > 500


def test_oracle_hints_edges():
    umem = np.zeros(4096, np.uint8)
    umem[0:16] = np.frombuffer(struct.pack("<QII", 5, 6, RX_TIME), np.uint8)
    umem[100:108] = np.frombuffer(struct.pack("<II", 9, RX_TIME), np.uint8)
    descs = np.zeros(4, xdpgpu.DESC_DTYPE)
    descs[0] = (16, 10, 0)        # the struct starts at the UMEM start
    descs[1] = (2, 10, 0)         # fewer than 4 bytes in front: no hints
    descs[2] = (108, 10, 0)       # rx_time id: the 16 bytes in front are its struct
    descs[3] = (8192, 10, 0)      # outside the UMEM
    got = oracle.hints(umem, descs, RX_TIME, MARK)
    assert tuple(got[0]) == (5, 6, RX_TIME)
    assert tuple(got[1]) == (0, 0, 0)
    assert got[2]["btf_id"] == RX_TIME and got[2]["value"] == 9
    assert tuple(got[3]) == (0, 0, 0)
    # ids of 0 never select a struct
    got = oracle.hints(umem, descs[:1], 0, 0)
    assert tuple(got[0]) == (0, 0, RX_TIME)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
def test_gpu_hints_vs_oracle(seed):
    torch = pytest.importorskip("torch")
    umem, descs, _ = hinted_pool(seed, n=20000)
    want = oracle.hints(umem, descs, RX_TIME, MARK)
    dev = torch.device("cuda:0")
    d_umem = torch.from_numpy(np.concatenate([umem, np.zeros(64, np.uint8)])).to(dev)
    d_desc = torch.from_numpy(descs.view(np.uint8)).to(dev)
    d_out = torch.full((len(descs) * 16,), 0xEE, dtype=torch.uint8, device=dev)
    with xdpgpu.XdpGpu(0) as g:
        g.hints_dev(d_umem, umem.nbytes, d_desc, len(descs), RX_TIME, MARK, d_out,
                    torch.cuda.current_stream())
        torch.cuda.synchronize()
    got = d_out.cpu().numpy().view(xdpgpu.HINTS_DTYPE)
    np.testing.assert_array_equal(got, want)
