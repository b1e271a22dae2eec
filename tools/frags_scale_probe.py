#!/usr/bin/env python3
# SPDX-License-Identifier: GPL-2.0
"""bench.py's multi-buffer leg (frags_run) at two packet counts: how much of
a launch over 65 536 jumbo packets is fixed cost (rocprofv3 --kernel-trace
--stats of it splits the launch by kernel)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bpf-examples_amd"))

import bench  # noqa: E402
import torch  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
st = torch.cuda.Stream(dev)
for n in (int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "65536,262144").split(",")):
    print(json.dumps(bench.frags_run(dev, st, n, 10, 0)), flush=True)
