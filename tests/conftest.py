# SPDX-License-Identifier: GPL-2.0
import os
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
for p in (os.path.join(ROOT, "bpf-examples_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")


_hostreg = None


@pytest.fixture(autouse=True)
def _gpu_drain(request):
    """A GPU test ends with the device drained and a fresh allocation used,
    so that an asynchronously reported device error fails the test whose
    kernels raised it, not the next one."""
    global _hostreg
    if os.environ.get("XDPGPU_HOSTREG_PROBE") == "1" and \
            request.node.get_closest_marker("gpu") is not None:
        # diagnostic: the runtime's host registrations per test (tests/hostreg.py)
        if _hostreg is None:
            import hostreg
            import test_gpu_parity
            import xdpgpu
            hostreg.install(xdpgpu, test_gpu_parity)
            _hostreg = hostreg
        _hostreg.current_test = request.node.nodeid
    yield
    if _hostreg is not None:
        _hostreg.end_of_test()
    if request.node.get_closest_marker("gpu") is None:
        return
    torch = sys.modules.get("torch")
    if torch is None or not torch.cuda.is_initialized():
        return
    torch.cuda.synchronize()
    probe = torch.zeros(4096, dtype=torch.uint8, device="cuda:0")
    probe.add_(1)
    assert int(probe.sum().item()) == 4096
    torch.cuda.synchronize()
    # a bounds-checked build (-DXDPGPU_DBG, tools/dbg_build.sh, selected with
    # XDPGPU_LIB): every access the RX kernels clamped is a failure of the
    # test that launched them (code -> [count, last value])
    xg = sys.modules.get("xdpgpu")
    lib = getattr(xg, "_lib", None) if xg else None
    if lib is not None and hasattr(lib, "xdpgpu_debug_read"):
        import ctypes
        import numpy as np
        dbg = np.zeros(64, np.uint64)
        assert lib.xdpgpu_debug_read(ctypes.c_void_p(dbg.ctypes.data)) == 0
        rec = {k: (int(dbg[2 * k]), hex(int(dbg[2 * k + 1])))
               for k in range(32) if dbg[2 * k]}
        assert not rec, f"bounds checks of the debug build fired: {rec}"


@pytest.fixture(scope="session")
def golden():
    import json
    import numpy as np
    d = os.path.join(ROOT, "tests", "golden")
    fx = dict(np.load(os.path.join(d, "fixtures.npz")))
    with open(os.path.join(d, "fixtures.json")) as f:
        meta = json.load(f)
    return fx, meta
