# SPDX-License-Identifier: GPL-2.0
"""Multi-GPU sharding of the packet pool (BASELINE config 5).

Every frame is independent, so the pool splits into contiguous descriptor
ranges, one per rank (one process per GPU, one xdpgpu context per process),
with no collective on the data path.  The only cross-rank traffic is the
end-of-run reduction of the counter block (xdpgpu_stats: frames, bytes,
verdict histogram, bad checksums) and of the timing (max over ranks), both a
few hundred bytes.  With the "nccl" backend that is RCCL over xGMI; the CPU
tests run the same code over "gloo".
"""
from __future__ import annotations

from typing import Dict, Tuple

STAT_KEYS = ("frames", "bytes", "l3_bad", "l4_bad", "l4_absent", "frag")
VERDICT_NAMES = ("ABORTED", "DROP", "PASS", "TX", "REDIRECT")


def shard_range(total: int, world: int, rank: int) -> Tuple[int, int]:
    """[lo, hi) of rank's contiguous share of total descriptors:
    [k*N/G, (k+1)*N/G)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} of {world}")
    return total * rank // world, total * (rank + 1) // world


def shard_seed(base: int, rank: int) -> int:
    """Pool seed of a rank's shard (config 5: config-2 content, seed offset
    by shard)."""
    return (base + rank) & 0xFFFFFFFFFFFFFFFF


def stats_vector(st: Dict) -> list:
    return [int(st[k]) for k in STAT_KEYS] + [int(st["verdict"][v]) for v in VERDICT_NAMES]


def stats_from_vector(vec) -> Dict:
    vals = [int(x) for x in vec]
    out = {k: vals[i] for i, k in enumerate(STAT_KEYS)}
    out["verdict"] = {v: vals[len(STAT_KEYS) + i] for i, v in enumerate(VERDICT_NAMES)}
    return out


def reduce_stats(st: Dict, device=None) -> Dict:
    """Sum a rank's counter block over all ranks (all_reduce SUM)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor(stats_vector(st), dtype=torch.int64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return stats_from_vector(t.cpu().tolist())


def reduce_timing(seconds: float, frames: int, ok: bool, device=None):
    """(max seconds, total frames, all ok) over ranks: the whole-job rate is
    total frames / max seconds (bench.py)."""
    import torch
    import torch.distributed as dist
    w = torch.tensor([seconds], dtype=torch.float64, device=device)
    f = torch.tensor([float(frames)], dtype=torch.float64, device=device)
    k = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(w, op=dist.ReduceOp.MAX)
        dist.all_reduce(f, op=dist.ReduceOp.SUM)
        dist.all_reduce(k, op=dist.ReduceOp.MIN)
    return float(w.item()), float(f.item()), bool(k.item() > 0)
