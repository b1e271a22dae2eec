# SPDX-License-Identifier: GPL-2.0
"""One rank of the multi-GPU path on a real device (launched by
tests/test_shard.py::test_two_rank_device_shards through torch.distributed.run,
two ranks sharing cuda:0 on the one-GPU box, gloo for the control
collectives): the rank generates its config-5 shard (config-2 content, seed
offset by rank, shard.py), runs it through the C ABI on the device
(xdpgpu_process_dev, its own context and stream), compares every frame with
the oracle, and reduces counters and timing exactly as bench.py does.
Rank 0 writes the reduced result to argv[1] as JSON; the exit status is
non-zero on any mismatch."""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (os.path.join(ROOT, "bpf-examples_amd"), os.path.join(ROOT, "oracle"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import oracle  # noqa: E402
import shard  # noqa: E402
import xdpgpu  # noqa: E402

FRAMES_PER_RANK = 1 << 18


def main(out_path: str) -> int:
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    n = FRAMES_PER_RANK
    umem, descs, _ = xdpgpu.pool_generate(n, xdpgpu.POOL_UDP4, 64,
                                          shard.shard_seed(0x5EED0005, rank))
    d_umem = torch.zeros(umem.nbytes + 64, dtype=torch.uint8, device=dev)
    d_umem[: umem.nbytes].copy_(torch.from_numpy(umem))
    dd = np.ascontiguousarray(descs, xdpgpu.DESC_DTYPE).view(np.uint8)
    d_desc = torch.from_numpy(dd.copy()).to(dev)
    d_v = torch.empty(n, dtype=torch.uint8, device=dev)
    d_res = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    d_tup = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    stream = torch.cuda.Stream(dev)
    with xdpgpu.XdpGpu(0, xdpgpu.CFG_DEFAULT | xdpgpu.CFG_STATS, 0, xdpgpu.TUPLE_V4) as ctx:
        dist.barrier()
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record(stream)
        ctx.process_dev(d_umem, umem.nbytes, d_desc, n, d_v, d_res, d_tup, stream=stream)
        t1.record(stream)
        torch.cuda.synchronize()
        st = ctx.stats()
    v = d_v.cpu().numpy()
    res = d_res.cpu().numpy().view(xdpgpu.RESULT_DTYPE)
    tup = d_tup.cpu().numpy()
    ov, ores, otup, ost = oracle.process(umem.copy(), descs, xdpgpu.CFG_DEFAULT, 0, 1)
    ok = (np.array_equal(v, ov) and res.tobytes() == ores.tobytes()
          and tup.tobytes() == otup.tobytes())
    ost = dict(ost)
    ost["verdict"] = dict(zip(shard.VERDICT_NAMES, ost["verdict"]))
    dev_tot = shard.reduce_stats(st)
    ora_tot = shard.reduce_stats(ost)
    secs, frames, all_ok = shard.reduce_timing(t0.elapsed_time(t1) * 1e-3, n, ok)
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump({"world": world, "frames": frames, "seconds_max": secs, "all_ok": all_ok,
                       "device_stats": dev_tot, "oracle_stats": ora_tot}, f)
    dist.barrier()
    dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
