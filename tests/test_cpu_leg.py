# SPDX-License-Identifier: GPL-2.0
"""The lean CPU leg of bench.py's cpu_baseline (oracle/cpu_leg.c) against the
oracle: verdicts, records, tuples and counters bit-exact on every pool kind
and configuration, and the golden fixtures; the calibration probes run."""
import json
import os

import numpy as np
import pytest

import oracle
import xdpgpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
CFGS = [(0x5, 0, 1), (0x5, 0x9E3779B9, 2), (0x4, 7, 1), (0x1, 0, 0), (0x5, 0, 0)]


def assert_leg_equal(umem, descs, flags, iv, fmt, what):
    ov, ores, otup, ost = oracle.process(umem.copy(), descs, flags, iv, fmt)
    lv, lres, ltup, lst, nfast = oracle.leg_process(umem.copy(), descs, flags, iv, fmt)
    bad = np.nonzero(ov != lv)[0]
    assert len(bad) == 0, f"{what}: verdicts differ at {bad[:8]}"
    bad = np.nonzero(ores.view(np.uint8).reshape(-1, 16) != lres.view(np.uint8).reshape(-1, 16))[0]
    assert len(bad) == 0, f"{what}: records differ at frames {np.unique(bad)[:8]}"
    if fmt:
        assert otup.tobytes() == ltup.tobytes(), f"{what}: tuples differ"
    assert ost == lst, f"{what}: counters differ"
    return nfast


@pytest.mark.parametrize("flags,iv,fmt", CFGS)
@pytest.mark.parametrize("kind,size,n", [(xdpgpu.POOL_UDP4, 64, 1 << 18),
                                         (xdpgpu.POOL_UDP4, 1500, 1 << 15),
                                         (xdpgpu.POOL_IMIX, 64, 1 << 16)],
                         ids=["udp64", "udp1500", "imix"])
def test_leg_vs_oracle_pools(kind, size, n, flags, iv, fmt):
    umem, descs, _ = xdpgpu.pool_generate(n, kind, size, 0x5EED0031)
    nfast = assert_leg_equal(umem, descs, flags, iv, fmt, f"pool {kind}/{size}")
    assert nfast > n // 2, "most frames take the leg's own path"


def test_leg_vs_oracle_tcp_vlan_odd():
    """TCP, VLAN-tagged and odd-length frames, and the over-read byte past
    the UMEM end: a pool at an odd base and one whose last frame ends the
    UMEM."""
    umem, descs, _ = xdpgpu.pool_generate(1 << 14, xdpgpu.POOL_IMIX, 64, 0x5EED0032)
    for flags, iv, fmt in CFGS:
        assert_leg_equal(umem, descs, flags, iv, fmt, "imix")
    # cut the UMEM right after the last frame: udp_csum's over-read byte
    # of an odd-length last datagram is then past the end (reads 0)
    last = int(np.argmax(descs["addr"]))
    end = int(descs["addr"][last]) + int(descs["len"][last])
    assert_leg_equal(np.ascontiguousarray(umem[:end]), descs, 0x5, 0, 1, "cut umem")


def test_leg_vs_golden_fixtures(golden):
    fx, meta = golden
    descs = fx["descs"].view(xdpgpu.DESC_DTYPE)
    for cfg in ("verify", "noverify"):
        flags, iv, fmt = meta["cfgs"][cfg]
        lv = oracle.leg_process(fx["umem"].copy(), descs, flags, iv, fmt)[0]
        np.testing.assert_array_equal(lv, fx[f"{cfg}_verdict"], err_msg=cfg)


def test_leg_bench_and_probe_run():
    umem, descs, _ = xdpgpu.pool_generate(1 << 15, xdpgpu.POOL_UDP4, 64, 0x5EED0033)
    dt, (v, res, tup) = oracle.leg_bench(umem, descs, 2, 2, True, 0x5, 0, 1)
    assert dt > 0
    ov = oracle.process(umem.copy(), descs, 0x5, 0, 1)[0]
    np.testing.assert_array_equal(v, ov)
    mine, ref = oracle.probe_pair(umem, descs, 2)
    assert mine > 0
    if os.path.isdir("/root/reference"):
        assert ref is not None and ref > 0


@pytest.mark.parametrize("flags,iv,fmt", [c for c in CFGS if c[2]])
@pytest.mark.parametrize("kind,size,n", [(xdpgpu.POOL_UDP4, 64, 1 << 16),
                                         (xdpgpu.POOL_UDP4, 1500, 1 << 13),
                                         (xdpgpu.POOL_IMIX, 64, 1 << 15)],
                         ids=["udp64", "udp1500", "imix"])
def test_reference_routine_leg_vs_oracle(kind, size, n, flags, iv, fmt):
    """The reference-routine leg (lib_checksum.h / jhash.h's own functions,
    oracle/ref_harness.c ref_leg_bench) gives the oracle's verdicts, records
    and tuples on every frame, and leaves the UMEM as it found it (the check
    words it zeroes are restored)."""
    if not os.path.isdir("/root/reference"):
        pytest.skip("reference tree absent (oracle/_ref is built from it)")
    umem, descs, _ = xdpgpu.pool_generate(n, kind, size, 0x5EED0034)
    u = umem.copy()
    r = oracle.ref_leg_bench(u, descs, 3, 2, False, flags, iv, fmt)
    assert r is not None
    dt, (v, res, tup) = r
    ov, ores, otup, _ = oracle.process(umem.copy(), descs, flags, iv, fmt)
    np.testing.assert_array_equal(v, ov)
    assert res.tobytes() == ores.tobytes()
    assert tup[: len(otup)].tobytes() == otup.tobytes()
    assert np.array_equal(u, umem)


def test_bench_cpu_baseline_is_the_reference_routines():
    """bench.py's cpu_baseline: with oracle/_ref present (built in this
    container), the value is the reference headers' routines' rate (kind
    "reference"), their outputs equal the port's, and the port's rate is
    reported beside it."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if not os.path.exists(os.path.join(root, "oracle", "_ref", "libref.so")):
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    sys.path.insert(0, root)
    import bench
    umem, descs, _ = xdpgpu.pool_generate(1 << 18, xdpgpu.POOL_UDP4, 64, 0x5EED0002)
    cb = bench.cpu_baseline(umem, descs, xdpgpu.CFG_DEFAULT, xdpgpu.TUPLE_V4, budget_s=0.2)
    assert cb["kind"] == "reference"
    assert cb["value"] == cb["reference_mpps"] > 0
    assert cb["port_mpps"] > 0 and cb["outputs_match_oracle"]
    assert cb["reference_outputs_match_leg"]
    json.dumps(cb)
