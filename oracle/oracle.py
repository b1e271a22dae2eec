# SPDX-License-Identifier: GPL-2.0
"""TEST INFRASTRUCTURE ONLY: ctypes binding of the parity oracle.

oracle/liboracle.so is the CPU restatement of the reference pipeline
(oracle/xdp_oracle.c).  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg import this module.  oracle/_ref/libref.so (reference
headers compiled in place) is optional and only exists where /root/reference
does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# XDPGPU_ORACLE_LIB: another build of the oracle (tools/asan.sh sanitized)
ORACLE_SO = os.environ.get("XDPGPU_ORACLE_LIB") or os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libref.so")

DESC_DTYPE = np.dtype([("addr", "<u8"), ("len", "<u4"), ("options", "<u4")])
RESULT_DTYPE = np.dtype([
    ("hash", "<u4"), ("l3_csum", "<u2"), ("l4_csum", "<u2"),
    ("flags", "u1"), ("l4_proto", "u1"), ("l3_off", "u1"), ("nvlan", "u1"),
    ("l4_off", "<u2"), ("l4_len", "<u2"),
])
TUPLE_BYTES = {0: 0, 1: 16, 2: 44}
NAT64_MAP_DTYPE = np.dtype([("v6", "u1", (16,)), ("v4", "<u4"), ("rsvd", "<u4")])


class Nat64Cfg(C.Structure):
    """struct xdpgpu_nat64_cfg (include/xdpgpu.h)"""
    _fields_ = [("v6_prefix", C.c_uint8 * 16), ("v6_plen", C.c_uint32),
                ("v4_prefix", C.c_uint32), ("v4_mask", C.c_uint32),
                ("allow_plen", C.c_uint32), ("allow_prefix", C.c_uint8 * 16),
                ("direction", C.c_uint32), ("flags", C.c_uint32),
                ("headroom", C.c_uint32), ("rsvd", C.c_uint32)]


class OStats(C.Structure):
    _fields_ = [("frames", C.c_uint64), ("bytes", C.c_uint64),
                ("verdict", C.c_uint64 * 5), ("l3_bad", C.c_uint64),
                ("l4_bad", C.c_uint64), ("l4_absent", C.c_uint64),
                ("frag", C.c_uint64), ("rsvd", C.c_uint64 * 5)]


_o = None
_r = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib() -> C.CDLL:
    global _o
    if _o is None:
        if not os.path.exists(ORACLE_SO):
            build()
        o = C.CDLL(ORACLE_SO)
        u8p, vp, u32, u64 = C.c_char_p, C.c_void_p, C.c_uint32, C.c_uint64
        o.oracle_do_csum.argtypes = [vp, C.c_int]
        o.oracle_do_csum.restype = u32
        o.oracle_ip_fast_csum.argtypes = [vp, C.c_uint]
        o.oracle_ip_fast_csum.restype = C.c_uint16
        o.oracle_csum_fold.argtypes = [u32]
        o.oracle_csum_fold.restype = C.c_uint16
        o.oracle_csum_tcpudp_nofold.argtypes = [u32, u32, u32, C.c_uint8, u32]
        o.oracle_csum_tcpudp_nofold.restype = u32
        o.oracle_csum_tcpudp_magic.argtypes = [u32, u32, u32, C.c_uint8, u32]
        o.oracle_csum_tcpudp_magic.restype = C.c_uint16
        o.oracle_udp_csum.argtypes = [u32, u32, u32, C.c_uint8, vp]
        o.oracle_udp_csum.restype = C.c_uint16
        o.oracle_csum_ipv6_magic.argtypes = [vp, vp, u32, C.c_uint8, u32]
        o.oracle_csum_ipv6_magic.restype = C.c_uint16
        o.oracle_csum_replace2.argtypes = [C.c_uint16, C.c_uint16, C.c_uint16]
        o.oracle_csum_replace2.restype = C.c_uint16
        o.oracle_jhash.argtypes = [vp, u32, u32]
        o.oracle_jhash.restype = u32
        o.oracle_jhash2.argtypes = [vp, u32, u32]
        o.oracle_jhash2.restype = u32
        o.oracle_jhash_3words.argtypes = [u32, u32, u32, u32]
        o.oracle_jhash_3words.restype = u32
        o.oracle_process.argtypes = [vp, u64, vp, u32, u32, u32, u32, vp, vp,
                                     vp, C.POINTER(OStats)]
        o.oracle_bench.argtypes = [vp, u64, vp, u32, u32, u32, u32, vp, vp,
                                   vp, u32, u32]
        o.oracle_bench.restype = C.c_double
        o.oracle_nat64.argtypes = [vp, u64, vp, u32, C.POINTER(Nat64Cfg), vp, u32,
                                   vp, vp]
        o.oracle_nat64_state_new.argtypes = [C.POINTER(Nat64Cfg), vp, u32, u64, u64]
        o.oracle_nat64_state_new.restype = vp
        o.oracle_nat64_state_free.argtypes = [vp]
        o.oracle_nat64_state_free.restype = None
        o.oracle_nat64_dyn.argtypes = [vp, u64, vp, u32, C.POINTER(Nat64Cfg), vp, u64,
                                       vp, vp]
        o.oracle_nat64_state_read.argtypes = [vp, vp, u32, C.POINTER(u32),
                                              C.POINTER(u64), vp, u32, C.POINTER(u32)]
        o.oracle_synproxy.argtypes = [vp, u64, vp, u32, vp, vp, vp, C.POINTER(u64)]
        o.oracle_hints.argtypes = [vp, u64, vp, u32, u32, u32, vp]
        o.oracle_v4addr_to_v6.argtypes = [vp, vp, vp, C.c_int]
        o.oracle_v6addr_to_v4.argtypes = [vp, C.c_int, vp, vp]
        del u8p
        _o = o
    return _o


def ref_lib() -> Optional[C.CDLL]:
    """The reference headers compiled in place, or None off this container."""
    global _r
    if _r is None:
        if not os.path.exists(REF_SO):
            if os.path.isdir("/root/reference"):
                build()
            if not os.path.exists(REF_SO):
                return None
        r = C.CDLL(REF_SO)
        vp, u32 = C.c_void_p, C.c_uint32
        r.ref_do_csum.argtypes = [vp, C.c_int]
        r.ref_do_csum.restype = u32
        r.ref_ip_fast_csum.argtypes = [vp, C.c_uint]
        r.ref_ip_fast_csum.restype = C.c_uint16
        r.ref_csum_fold.argtypes = [u32]
        r.ref_csum_fold.restype = C.c_uint16
        r.ref_csum_tcpudp_nofold.argtypes = [u32, u32, u32, C.c_uint8, u32]
        r.ref_csum_tcpudp_nofold.restype = u32
        r.ref_csum_tcpudp_magic.argtypes = [u32, u32, u32, C.c_uint8, u32]
        r.ref_csum_tcpudp_magic.restype = C.c_uint16
        r.ref_udp_csum.argtypes = [u32, u32, u32, C.c_uint8, vp]
        r.ref_udp_csum.restype = C.c_uint16
        r.ref_memset32_htonl.argtypes = [vp, u32, u32]
        r.ref_memset32_htonl.restype = None
        for name, n in (("ref_jhash", 3), ("ref_jhash2", 3)):
            f = getattr(r, name)
            f.argtypes = [vp, u32, u32]
            f.restype = u32
        r.ref_jhash_3words.argtypes = [u32, u32, u32, u32]
        r.ref_jhash_3words.restype = u32
        r.ref_jhash_2words.argtypes = [u32, u32, u32]
        r.ref_jhash_2words.restype = u32
        r.ref_jhash_1word.argtypes = [u32, u32]
        r.ref_jhash_1word.restype = u32
        r.ref_probe.argtypes = [vp, C.c_uint64, vp, u32, u32, C.POINTER(C.c_uint64)]
        r.ref_probe.restype = C.c_double
        r.ref_leg_bench.argtypes = [vp, C.c_uint64, vp, u32, u32, u32, u32, vp, vp, vp, u32,
                                    u32, C.c_int]
        r.ref_leg_bench.restype = C.c_double
        _r = r
    return _r


def buf(b: bytes):
    """A ctypes buffer holding b (kept alive by the caller)."""
    return C.create_string_buffer(bytes(b), len(b) + 8)


def process(umem: np.ndarray, descs: np.ndarray, flags: int = 0x5,
            initval: int = 0, tuple_fmt: int = 1):
    """Run the oracle pipeline: returns (verdict, res, tuples bytes, stats).

    umem is modified in place only for ICMPv6 echo rewrites (flag 0x2)."""
    o = lib()
    descs = np.ascontiguousarray(descs, DESC_DTYPE)
    n = len(descs)
    verdict = np.zeros(n, np.uint8)
    res = np.zeros(n, RESULT_DTYPE)
    tb = TUPLE_BYTES[tuple_fmt]
    tup = np.zeros(n * tb if tb else 1, np.uint8)
    st = OStats()
    rc = o.oracle_process(umem.ctypes.data, umem.nbytes, descs.ctypes.data, n,
                          flags, initval & 0xffffffff, tuple_fmt,
                          verdict.ctypes.data, res.ctypes.data,
                          tup.ctypes.data if tb else None, C.byref(st))
    if rc:
        raise RuntimeError(f"oracle_process rc={rc}")
    stats = {"frames": st.frames, "bytes": st.bytes,
             "verdict": list(st.verdict), "l3_bad": st.l3_bad,
             "l4_bad": st.l4_bad, "l4_absent": st.l4_absent, "frag": st.frag}
    return verdict, res, (tup[: n * tb] if tb else None), stats


def bench(umem: np.ndarray, descs: np.ndarray, threads: int, reps: int,
          flags: int = 0x1, initval: int = 0, tuple_fmt: int = 1) -> float:
    """Wall seconds for `reps` passes of the oracle over descs on `threads`."""
    o = lib()
    descs = np.ascontiguousarray(descs, DESC_DTYPE)
    n = len(descs)
    verdict = np.zeros(n, np.uint8)
    res = np.zeros(n, RESULT_DTYPE)
    tb = TUPLE_BYTES[tuple_fmt]
    tup = np.zeros(max(1, n * tb), np.uint8)
    return o.oracle_bench(umem.ctypes.data, umem.nbytes, descs.ctypes.data, n,
                          flags, initval, tuple_fmt, verdict.ctypes.data,
                          res.ctypes.data, tup.ctypes.data, threads, reps)


def nat64(umem: np.ndarray, descs: np.ndarray, cfg: "Nat64Cfg", smap: np.ndarray):
    """Run the nat64 oracle in place on umem: returns (action, out descs)."""
    o = lib()
    descs = np.ascontiguousarray(descs, DESC_DTYPE)
    smap = np.ascontiguousarray(smap, NAT64_MAP_DTYPE)
    n = len(descs)
    action = np.zeros(n, np.uint8)
    out = np.zeros(n, DESC_DTYPE)
    o.oracle_nat64(umem.ctypes.data, umem.nbytes, descs.ctypes.data, n, C.byref(cfg),
                   smap.ctypes.data if len(smap) else None, len(smap),
                   action.ctypes.data, out.ctypes.data)
    return action, out


NAT64_ENTRY_DTYPE = np.dtype([("v6", "u1", (16,)), ("v4", "<u4"), ("static_conf", "<u4"),
                              ("last_seen", "<u8")])


class Nat64State:
    """The nat64 state tables with dynamic allocation (oracle_nat64_state):
    one `run` is one batch at time `now`, frames in order."""

    def __init__(self, cfg: "Nat64Cfg", smap: np.ndarray, timeout_ns: int,
                 next_addr: int = 1):
        self.o = lib()
        self.cfg = cfg
        smap = np.ascontiguousarray(smap, NAT64_MAP_DTYPE)
        self.h = self.o.oracle_nat64_state_new(C.byref(cfg),
                                               smap.ctypes.data if len(smap) else None,
                                               len(smap), timeout_ns, next_addr)
        if not self.h:
            raise MemoryError("oracle_nat64_state_new")

    def run(self, umem: np.ndarray, descs: np.ndarray, now: int):
        descs = np.ascontiguousarray(descs, DESC_DTYPE)
        n = len(descs)
        action = np.zeros(n, np.uint8)
        out = np.zeros(n, DESC_DTYPE)
        self.o.oracle_nat64_dyn(umem.ctypes.data, umem.nbytes, descs.ctypes.data, n,
                                C.byref(self.cfg), self.h, now, action.ctypes.data,
                                out.ctypes.data)
        return action, out

    def state(self):
        """(entries in insertion order, next_addr, reclaim queue)"""
        n, nq, na = C.c_uint32(0), C.c_uint32(0), C.c_uint64(0)
        self.o.oracle_nat64_state_read(self.h, None, 0, C.byref(n), C.byref(na), None, 0,
                                       C.byref(nq))
        ent = np.zeros(n.value, NAT64_ENTRY_DTYPE)
        q = np.zeros(nq.value, np.uint32)
        self.o.oracle_nat64_state_read(self.h, ent.ctypes.data, n.value, C.byref(n),
                                       C.byref(na), q.ctypes.data, nq.value, C.byref(nq))
        return ent, int(na.value), q

    def close(self):
        if self.h:
            self.o.oracle_nat64_state_free(self.h)
            self.h = None

    def __del__(self):
        self.close()


def synproxy(umem: np.ndarray, descs: np.ndarray, cfg):
    """The SYN proxy oracle in place on umem: (verdict, out descs, synacks).
    cfg: xdpgpu.SynproxyCfg (the same C layout)."""
    descs = np.ascontiguousarray(descs, DESC_DTYPE)
    n = len(descs)
    verdict = np.zeros(n, np.uint8)
    out = np.zeros(n, DESC_DTYPE)
    cnt = C.c_uint64(0)
    lib().oracle_synproxy(umem.ctypes.data, umem.nbytes, descs.ctypes.data, n,
                          C.addressof(cfg), verdict.ctypes.data, out.ctypes.data,
                          C.byref(cnt))
    return verdict, out, int(cnt.value)


def hints(umem: np.ndarray, descs: np.ndarray, rx_time_id: int, mark_id: int):
    """XDP hints in front of each frame (xdpgpu_hints_dev semantics)."""
    import xdpgpu
    descs = np.ascontiguousarray(descs, DESC_DTYPE)
    out = np.zeros(len(descs), xdpgpu.HINTS_DTYPE)
    lib().oracle_hints(umem.ctypes.data, umem.nbytes, descs.ctypes.data, len(descs),
                       rx_time_id, mark_id, out.ctypes.data)
    return out


def v4addr_to_v6(a4: bytes, pref: bytes, plen: int):
    o = lib()
    out = C.create_string_buffer(16)
    ok = o.oracle_v4addr_to_v6(buf(a4), out, buf(pref), plen)
    return bytes(out.raw[:16]) if ok else None


def v6addr_to_v4(a6: bytes, plen: int):
    o = lib()
    a4 = C.create_string_buffer(4)
    pref = C.create_string_buffer(16)
    ok = o.oracle_v6addr_to_v4(buf(a6), plen, a4, pref)
    return (bytes(a4.raw[:4]), bytes(pref.raw[:16])) if ok else None


def _leg_lib() -> C.CDLL:
    o = lib()
    if not hasattr(o, "_leg_bound"):
        vp, u32, u64 = C.c_void_p, C.c_uint32, C.c_uint64
        o.cpu_leg_process.argtypes = [vp, u64, vp, u32, u32, u32, u32, vp, vp, vp, vp]
        o.cpu_leg_process.restype = u32
        o.cpu_leg_bench.argtypes = [vp, u64, vp, u32, u32, u32, u32, vp, vp, vp, u32, u32,
                                    C.c_int]
        o.cpu_leg_bench.restype = C.c_double
        o.cpu_leg_probe.argtypes = [vp, u64, vp, u32, u32, C.POINTER(C.c_uint64)]
        o.cpu_leg_probe.restype = C.c_double
        o._leg_bound = True
    return o


def leg_process(umem: np.ndarray, descs: np.ndarray, flags: int = 0x5,
                initval: int = 0, tuple_fmt: int = 1):
    """The lean CPU leg (oracle/cpu_leg.c): same outputs as process();
    also returns how many frames took its fast shape."""
    o = _leg_lib()
    descs = np.ascontiguousarray(descs, DESC_DTYPE)
    n = len(descs)
    verdict = np.zeros(n, np.uint8)
    res = np.zeros(n, RESULT_DTYPE)
    tb = TUPLE_BYTES[tuple_fmt]
    tup = np.zeros(n * tb if tb else 1, np.uint8)
    st = OStats()
    nfast = o.cpu_leg_process(umem.ctypes.data, umem.nbytes, descs.ctypes.data, n, flags,
                              initval, tuple_fmt, verdict.ctypes.data, res.ctypes.data,
                              tup.ctypes.data if tb else None, C.byref(st))
    stats = {"frames": st.frames, "bytes": st.bytes, "verdict": list(st.verdict),
             "l3_bad": st.l3_bad, "l4_bad": st.l4_bad, "l4_absent": st.l4_absent,
             "frag": st.frag}
    return verdict, res, tup, stats, nfast


def leg_bench(umem: np.ndarray, descs: np.ndarray, threads: int, reps: int, pin: bool,
              flags: int = 0x5, initval: int = 0, tuple_fmt: int = 1):
    """Wall seconds for `reps` passes of the lean leg over descs on
    `threads` threads (pinned to the affinity set's CPUs when pin), and the
    outputs of the last pass."""
    o = _leg_lib()
    descs = np.ascontiguousarray(descs, DESC_DTYPE)
    n = len(descs)
    verdict = np.zeros(n, np.uint8)
    res = np.zeros(n, RESULT_DTYPE)
    tb = TUPLE_BYTES[tuple_fmt]
    tup = np.zeros(max(1, n * tb), np.uint8)
    dt = o.cpu_leg_bench(umem.ctypes.data, umem.nbytes, descs.ctypes.data, n, flags,
                         initval, tuple_fmt, verdict.ctypes.data, res.ctypes.data,
                         tup.ctypes.data if tb else None, threads, reps, 1 if pin else 0)
    return dt, (verdict, res, tup)


def ref_leg_bench(umem: np.ndarray, descs: np.ndarray, threads: int, reps: int, pin: bool,
                  flags: int = 0x5, initval: int = 0, tuple_fmt: int = 1):
    """As leg_bench, with the reference headers' own checksum and hash
    routines (oracle/ref_harness.c ref_leg_bench); None off this container
    or when oracle/_ref was not built.  umem is written (check words zeroed
    and restored), so pass a copy when it is shared."""
    r = ref_lib()
    if r is None:
        return None
    descs = np.ascontiguousarray(descs, DESC_DTYPE)
    n = len(descs)
    verdict = np.zeros(n, np.uint8)
    res = np.zeros(n, RESULT_DTYPE)
    tb = TUPLE_BYTES[tuple_fmt]
    tup = np.zeros(max(1, n * tb), np.uint8)
    dt = r.ref_leg_bench(umem.ctypes.data, umem.nbytes, descs.ctypes.data, n, flags, initval,
                         tuple_fmt, verdict.ctypes.data, res.ctypes.data,
                         tup.ctypes.data if tb else None, threads, reps, 1 if pin else 0)
    return dt, (verdict, res, tup)


def probe_pair(umem: np.ndarray, descs: np.ndarray, reps: int):
    """Seconds of the survey probe's work (parse, IPv4 and UDP checksums,
    13-byte jhash) per pass on one thread: (this leg's arithmetic, the
    reference headers' routines or None off this container)."""
    o = _leg_lib()
    descs = np.ascontiguousarray(descs, DESC_DTYPE)
    acc = C.c_uint64(0)
    mine = o.cpu_leg_probe(umem.ctypes.data, umem.nbytes, descs.ctypes.data, len(descs),
                           reps, C.byref(acc)) / reps
    r = ref_lib()
    ref = None
    if r is not None:
        ref = r.ref_probe(umem.ctypes.data, umem.nbytes, descs.ctypes.data, len(descs),
                          reps, C.byref(acc)) / reps
    return mine, ref
