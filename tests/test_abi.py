# SPDX-License-Identifier: GPL-2.0
"""CPU: the C-ABI library builds, loads and exports exactly what
include/xdpgpu.h declares; the host-only pool generator is deterministic and
its intended verdicts agree with the oracle.  No GPU compute here."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import oracle
import xdpgpu

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def header_functions():
    src = open(os.path.join(ROOT, "include", "xdpgpu.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(xdpgpu_\w+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    lib = xdpgpu.load_library()
    declared = header_functions()
    assert declared, "no declarations parsed"
    assert sorted(xdpgpu.EXPORTS) == declared
    for name in declared:
        assert hasattr(lib, name), f"{name} missing from libxdpgpu.so"


def test_library_contains_gfx950_code_object():
    blob = open(xdpgpu.LIB_PATH, "rb").read()
    assert b"gfx950" in blob
    assert b"xdp_rx_db_kernel" in blob


def test_abi_version_and_struct_sizes():
    lib = xdpgpu.load_library()
    assert lib.xdpgpu_abi_version() == 1
    assert C.sizeof(xdpgpu.Cfg) == 32
    assert C.sizeof(xdpgpu.Stats) == 8 * 16
    assert xdpgpu.RESULT_DTYPE.itemsize == 16


def test_init_without_gpu_fails_loudly():
    if xdpgpu.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(xdpgpu.XdpGpuError):
        xdpgpu.XdpGpu(0)


@pytest.mark.parametrize("kind,size", [(xdpgpu.POOL_UDP4, 64), (xdpgpu.POOL_UDP4, 1500),
                                       (xdpgpu.POOL_IMIX, 64)])
def test_pool_deterministic_across_threads(kind, size):
    a = xdpgpu.pool_generate(70000, kind, size, 0x5EED0002, threads=1)
    b = xdpgpu.pool_generate(70000, kind, size, 0x5EED0002, threads=7)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("kind,size,seed", [(xdpgpu.POOL_UDP4, 64, 0x5EED0002),
                                            (xdpgpu.POOL_UDP4, 1500, 0x5EED0002),
                                            (xdpgpu.POOL_IMIX, 64, 0x5EED0003)])
def test_pool_intent_matches_oracle(kind, size, seed):
    umem, descs, expect = xdpgpu.pool_generate(100000, kind, size, seed)
    v, res, tup, st = oracle.process(umem, descs, 0x5)
    np.testing.assert_array_equal(v, expect)
    # every verdict class the survey asks for is exercised
    counts = np.bincount(v, minlength=5)
    assert counts[xdpgpu.ABORTED] and counts[xdpgpu.DROP] and counts[xdpgpu.PASS]
    assert counts[xdpgpu.REDIRECT] > 0.9 * len(v)


def test_pool_imix_mix():
    umem, descs, expect = xdpgpu.pool_generate(120000, xdpgpu.POOL_IMIX, 64, 0x5EED0003)
    v, res, tup, st = oracle.process(umem, descs, 0x5, 0, 2)
    sizes = np.bincount(np.searchsorted([64, 570, 1500], descs["len"]), minlength=3)
    frac = sizes / sizes.sum()
    assert abs(frac[0] - 7 / 12) < 0.03 and abs(frac[2] - 1 / 12) < 0.02
    live = (v == xdpgpu.REDIRECT)
    f = res["flags"][live]
    # 30 % of the pool IPv6, all in the 570/1500 B classes
    assert 0.27 < np.mean((f & xdpgpu.F_IPV6) > 0) < 0.33
    big = descs["len"][live] > 64
    assert not ((f & xdpgpu.F_IPV6) > 0)[~big].any()
    assert 0.17 < np.mean((f & xdpgpu.F_VLAN) > 0) < 0.27
    # the round-2 mix (30 % of the 570/1500 B classes) stays available
    umem, descs, _ = xdpgpu.pool_generate(120000, xdpgpu.POOL_IMIX, 64, 0x5EED0003,
                                          ppm_v6=125000)
    v, res, _, _ = oracle.process(umem, descs, 0x5, 0, 2)
    f = res["flags"][v == xdpgpu.REDIRECT]
    assert 0.10 < np.mean((f & xdpgpu.F_IPV6) > 0) < 0.15


def test_reference_generator_frames():
    # xdpsock -s 64 base frame, SURVEY.md §8c golden bytes
    umem, descs, _ = xdpgpu.pool_generate(4, xdpgpu.POOL_XDPSOCK, 64)
    f = umem[descs[0]["addr"]:descs[0]["addr"] + 60].tobytes()
    assert f.hex() == ("3cfdfe9e7f71ecb1d7983ac008004500002e000000004011527c0a0a0a100a0a"
                       "0a2010001000001a0291123456781234567812345678123456781234")
    assert descs[0]["len"] == 60
    umem, descs, _ = xdpgpu.pool_generate(2, xdpgpu.POOL_XDPSOCK, 64, vlan=1)
    f = umem[descs[0]["addr"]:descs[0]["addr"] + 60].tobytes()
    assert f[28:30].hex() == "5280" and f[44:46].hex() == "6b45"
    umem, descs, _ = xdpgpu.pool_generate(2, xdpgpu.POOL_XDPSOCK, 1500)
    f = umem[descs[0]["addr"]:descs[0]["addr"] + 60].tobytes()
    assert f[24:26].hex() == "4ce0" and f[40:42].hex() == "2d92"
    umem, descs, _ = xdpgpu.pool_generate(2, xdpgpu.POOL_AFXDP_USER, 64)
    f = umem[descs[0]["addr"]:descs[0]["addr"] + 64].tobytes()
    assert f[24:26].hex() == "a16a" and f[40:42].hex() == "b308"
    assert descs[0]["len"] == 64
