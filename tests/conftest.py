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


@pytest.fixture(scope="session")
def golden():
    import json
    import numpy as np
    d = os.path.join(ROOT, "tests", "golden")
    fx = dict(np.load(os.path.join(d, "fixtures.npz")))
    with open(os.path.join(d, "fixtures.json")) as f:
        meta = json.load(f)
    return fx, meta
