#!/usr/bin/env python3
# SPDX-License-Identifier: GPL-2.0
"""One of bench.py's in-place legs alone (no config-2 leg before it): for
rocprofv3 --pmc passes over that leg's kernel (tools/pmc_profile.sh,
PMC_CMD), whose summary bench.py attaches to the leg's line.

    python3 tools/leg_probe.py --leg echo|synproxy [--steps K]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bpf-examples_amd"))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--leg", choices=("echo", "synproxy"), required=True)
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream(dev)
    fn = bench.echo_run if args.leg == "echo" else bench.synproxy_run
    print(json.dumps(fn(dev, stream, 8 << 20, args.steps, 0)), flush=True)


if __name__ == "__main__":
    main()
