# SPDX-License-Identifier: GPL-2.0
"""CPU: the oracle is pinned to the reference (golden vectors, KATs and, where
/root/reference exists, the reference headers compiled in place)."""
import ctypes as C
import os

import numpy as np
import pytest

import oracle

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def o():
    return oracle.lib()


def test_jhash_kats(o):
    # include/jhash.h (lookup3 hashlittle) known answers, SURVEY.md §8a a-J1/J2
    s = b"Four score and seven years ago"
    assert o.oracle_jhash(b"", 0, 0) == 0xDEADBEEF
    assert o.oracle_jhash(b"", 0, 0xDEADBEEF) == 0xBD5B7DDE
    assert o.oracle_jhash(s, 30, 0) == 0x17770551
    assert o.oracle_jhash(s, 30, 1) == 0xCD628161
    assert o.oracle_jhash(bytes(44), 44, 0) == 0xB0B6DC57
    assert o.oracle_jhash(bytes(range(44)), 44, 0) == 0x3A104DF7
    assert o.oracle_jhash2(bytes(range(44)), 11, 0) == 0x3A104DF7
    assert o.oracle_jhash_3words(1, 2, 3, 0) == 0xA46158F5


def test_jhash_vectors(o):
    v = np.load(os.path.join(GOLD, "jhash_vectors.npz"))
    for k in range(len(v["klen"])):
        key = v["keys"][k].tobytes()
        assert o.oracle_jhash(key, int(v["klen"][k]), int(v["initval"][k])) == v["jhash"][k]
    for k in range(len(v["wlen"])):
        key = v["keys"][k].tobytes()
        assert o.oracle_jhash2(key, int(v["wlen"][k]), int(v["initval"][k])) == v["jhash2"][k]
    for k in range(len(v["words3"])):
        a, b, c = (int(x) for x in v["words3"][k])
        assert o.oracle_jhash_3words(a, b, c, int(v["initval"][k])) == v["jhash_3words"][k]
        # jhash_2words(a, b, iv) = jhash_3words(a, b, 0, iv - 4), jhash_1word
        # likewise (jhash.h:157-170: initval + JHASH_INITVAL + 4 nwords)
        iv = int(v["initval"][k])
        assert o.oracle_jhash_3words(a, b, 0, (iv - 4) & 0xffffffff) == v["jhash_2words"][k]
        assert o.oracle_jhash_3words(a, 0, 0, (iv - 8) & 0xffffffff) == v["jhash_1word"][k]


def test_csum_vectors(o):
    v = np.load(os.path.join(GOLD, "csum_vectors.npz"))
    raw = C.create_string_buffer(v["buf"].tobytes(), len(v["buf"]) + 16)
    base = C.addressof(raw)
    for off, ln, want in zip(v["offs"], v["lens"], v["do_csum"]):
        assert o.oracle_do_csum(base + int(off), int(ln)) == want
    for k in range(len(v["ihl"])):
        assert o.oracle_ip_fast_csum(v["hdrs"][k].tobytes(), int(v["ihl"][k])) == \
            v["ip_fast_csum"][k]
    for k in range(len(v["udp_len"])):
        assert o.oracle_udp_csum(int(v["saddr"][k]), int(v["daddr"][k]),
                                 int(v["udp_len"][k]), int(v["proto"][k]),
                                 v["udp_data"][k].tobytes()) == v["udp_csum"][k]
        assert o.oracle_csum_tcpudp_magic(int(v["saddr"][k]), int(v["daddr"][k]),
                                          int(v["udp_len"][k]), int(v["proto"][k]),
                                          int(v["sums"][k])) == v["tcpudp_magic"][k]
    for s, want in zip(v["sums"], v["csum_fold"]):
        assert o.oracle_csum_fold(int(s)) == want


def test_survey_golden_frame(o):
    # xdpsock default 60-byte frame with the reference's checksums
    f = bytes.fromhex(
        "3cfdfe9e7f71ecb1d7983ac008004500002e000000004011527c0a0a0a100a0a"
        "0a2010001000001a0291123456781234567812345678123456781234")
    assert o.oracle_ip_fast_csum(f[14:34], 5) == 0
    hdr = bytearray(f[14:34])
    hdr[10] = hdr[11] = 0
    assert o.oracle_ip_fast_csum(bytes(hdr), 5) == 0x7C52
    seg = bytearray(f[34:60] + b"\0")
    seg[6] = seg[7] = 0
    sa = int.from_bytes(f[26:30], "little")
    da = int.from_bytes(f[30:34], "little")
    assert o.oracle_udp_csum(sa, da, 26, 17, bytes(seg)) == 0x9102


def test_csum_replace2(o):
    # af_xdp_user.c:590-606, incremental update of an echo request
    for s in (0x0000, 0xFFFF, 0x1234, 0x0080, 0x7F7F):
        got = o.oracle_csum_replace2(s, 0x0080, 0x0081)
        # one's complement identity: ~new = ~old_sum - old + new (mod 0xffff)
        a = (~s & 0xFFFF) + (~0x0080 & 0xFFFF) + 0x0081
        while a >> 16:
            a = (a & 0xFFFF) + (a >> 16)
        assert got == (~a & 0xFFFF)


@pytest.mark.parametrize("cfg", ["verify", "echo_net", "noverify"])
def test_oracle_matches_fixtures(golden, cfg):
    fx, meta = golden
    flags, iv, fmt = meta["cfgs"][cfg]
    umem = fx["umem"].copy()
    descs = fx["descs"].view(oracle.DESC_DTYPE)
    v, res, tup, st = oracle.process(umem, descs, flags, iv, fmt)
    np.testing.assert_array_equal(v, fx[f"{cfg}_verdict"])
    np.testing.assert_array_equal(res.view(np.uint8), fx[f"{cfg}_res"])
    np.testing.assert_array_equal(tup, fx[f"{cfg}_tup"])
    np.testing.assert_array_equal(umem, fx[f"{cfg}_umem_after"])
    if cfg == "verify":
        assert list(v) == meta["expected_verdict_verify"]


def test_oracle_against_reference_headers_random():
    """Where the reference tree exists: oracle primitives == reference
    headers on fresh random inputs (not only the committed vectors)."""
    r = oracle.ref_lib()
    if r is None:
        pytest.skip("reference tree not present (GPU box)")
    o = oracle.lib()
    rng = np.random.default_rng()
    buf = rng.integers(0, 256, 20000, dtype=np.uint8).tobytes()
    raw = C.create_string_buffer(buf, len(buf) + 16)
    base = C.addressof(raw)
    for _ in range(3000):
        off = int(rng.integers(0, 16))
        ln = int(rng.integers(0, 9000))
        assert o.oracle_do_csum(base + off, ln) == r.ref_do_csum(base + off, ln)
    for _ in range(2000):
        ln = int(rng.integers(0, 100))
        iv = int(rng.integers(0, 2 ** 32))
        k = rng.integers(0, 256, 100, dtype=np.uint8).tobytes()
        assert o.oracle_jhash(k, ln, iv) == r.ref_jhash(oracle.buf(k), ln, iv)
