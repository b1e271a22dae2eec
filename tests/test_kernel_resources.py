# SPDX-License-Identifier: GPL-2.0
"""The product library's gfx950 kernels keep everything in registers: no
kernel has scratch (private segment) or VGPR spills, read from the code
object's AMDGPU metadata (tools/kres.py; CPU only, no GPU).  A scratch load
in a tile loop that has LDS-DMA in flight costs the compiler's vmcnt(0), a
full drain of the loop's prefetch."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import kres  # noqa: E402

pytestmark = pytest.mark.skipif(not os.path.exists(kres.READELF) or
                                not os.path.exists(kres.LIB),
                                reason="llvm-readelf or the built library missing")


def test_no_scratch_or_vgpr_spills():
    ks = kres.kernels()
    # every translation unit's code object (one offload bundle each)
    for part in ("xdp_rx_db_kernel", "xdp_nat64_kernel", "xdp_nat64_fast_kernel",
                 "synproxy_kernel", "frag_count_kernel", "hints_kernel",
                 "echo_writeback_kernel", "umem_gather_kernel"):
        assert any(part in k for k in ks), part
    bad = {k: v for k, v in ks.items() if v["scratch"] or v["vgpr_spill"]}
    assert not bad, f"kernels with scratch or VGPR spills: {bad}"


def test_rx_instances_occupancy():
    """The per-CU RX kernel: 15 waves on one block per CU, so at most 128
    VGPRs (4 waves on a SIMD) and the CU's LDS for the waves' buffers."""
    ks = kres.kernels()
    rx = {k: v for k, v in ks.items() if "xdp_rx_db_kernel" in k}
    assert len(rx) >= 5
    for k, v in rx.items():
        assert v["vgpr"] <= 128, (k, v)


def test_nat64_general_kernel_occupancy():
    """nat64's general kernel, the reference's translation, is held to 4
    waves a SIMD with its headers in registers (csrc/nat64.hip
    __launch_bounds__)."""
    ks = kres.kernels()
    gen = {k: v for k, v in ks.items() if "xdp_nat64_kernelILb0E" in k}
    assert gen
    for k, v in gen.items():
        assert v["vgpr"] <= 128 and not v["scratch"], (k, v)
