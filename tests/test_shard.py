# SPDX-License-Identifier: GPL-2.0
"""The N > 1 path on CPU: two gloo ranks, each owning a contiguous shard of
one pool (shard.py), process it (oracle as the stand-in for the device
path: these tests check the split and the reductions, not the kernels) and
reduce counters and timing as bench.py does.  The reduced counters must
equal one pass over the whole pool."""
import os
import socket

import numpy as np
import pytest

import oracle
import shard
import xdpgpu

torch = pytest.importorskip("torch")

N_TOTAL = 20011            # odd: ranks get unequal shares


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_main(rank, world, port, out_dir):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    umem, descs, _ = xdpgpu.pool_generate(N_TOTAL, xdpgpu.POOL_IMIX, 64, 0x5EED0003)
    lo, hi = shard.shard_range(N_TOTAL, world, rank)
    _, _, _, st = oracle.process(umem.copy(), np.ascontiguousarray(descs[lo:hi]), 0x5, 0, 1)
    st = dict(st)
    st["verdict"] = dict(zip(shard.VERDICT_NAMES, st["verdict"]))
    tot = shard.reduce_stats(st)
    secs, frames, ok = shard.reduce_timing(0.5 + rank, hi - lo, rank != 7)
    if rank == 0:
        np.save(os.path.join(out_dir, "tot.npy"), np.array(shard.stats_vector(tot)))
        np.save(os.path.join(out_dir, "timing.npy"), np.array([secs, frames, ok]))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range_covers_pool():
    for world in (1, 2, 3, 8):
        spans = [shard.shard_range(N_TOTAL, world, r) for r in range(world)]
        assert spans[0][0] == 0 and spans[-1][1] == N_TOTAL
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
        sizes = [h - l for l, h in spans]
        assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard.shard_range(10, 2, 2)


def test_two_rank_gloo_reduction(tmp_path):
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    got = shard.stats_from_vector(np.load(tmp_path / "tot.npy"))
    umem, descs, _ = xdpgpu.pool_generate(N_TOTAL, xdpgpu.POOL_IMIX, 64, 0x5EED0003)
    _, _, _, want = oracle.process(umem.copy(), descs, 0x5, 0, 1)
    for k in shard.STAT_KEYS:
        assert got[k] == want[k], k
    assert [got["verdict"][v] for v in shard.VERDICT_NAMES] == want["verdict"]
    secs, frames, ok = np.load(tmp_path / "timing.npy")
    assert secs == 1.5 and frames == N_TOTAL and ok == 1.0


def _torchrun(script_args, env_extra=None, timeout=240):
    import subprocess
    import sys
    env = dict(os.environ)
    env.update(env_extra or {})
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}"] + script_args
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env,
                          cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


@pytest.mark.gpu
def test_two_rank_device_shards(tmp_path):
    """The N > 1 path on the device: two ranks (one process each, as
    bench.py runs under torch.distributed.run), each with its own context on
    cuda:0 and its config-5 shard, every frame compared with the oracle on
    each rank; counters and timing reduced over gloo as bench.py reduces
    them over RCCL, and the reduced device counters equal the reduced
    oracle counters (tests/shard_worker.py)."""
    import json
    out = tmp_path / "shards.json"
    r = _torchrun([os.path.join("tests", "shard_worker.py"), str(out)])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    js = json.loads(out.read_text())
    assert js["world"] == 2 and js["all_ok"] is True
    assert js["frames"] == 2 * (1 << 18) and js["seconds_max"] > 0
    assert js["device_stats"] == js["oracle_stats"]
    assert js["device_stats"]["frames"] == 2 * (1 << 18)


@pytest.mark.gpu
def test_bench_two_rank_rehearsal():
    """bench.py's own N-rank path (torchrun launch, set_device before the
    process group, per-rank shards with offset seeds, barrier-bracketed
    timing, max-over-ranks reduction, one rank-0 line), two ranks sharing
    cuda:0 (XDPGPU_BENCH_REHEARSE=1: gloo for the three control scalars):
    the rank-0 line reports both ranks' frames and correct verdicts."""
    import json
    r = _torchrun(["bench.py", "--gpus", "2", "--frames", str(1 << 20), "--steps", "3",
                   "--warmup", "1", "--no-cpu", "--no-secondary"],
                  {"XDPGPU_BENCH_REHEARSE": "1"})
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    js = json.loads(lines[0])
    assert js["n_gpus"] == 2 and js["verdicts_ok"] is True and js["value"] > 0
    assert js["scaling"] == "weak" and js["config"]["parallelism"] == "shard2"
    assert js["config"]["frames_per_gpu"] == 1 << 20


@pytest.mark.gpu
def test_bench_self_launch():
    """`python bench.py --gpus 2` with no outer launcher, as the driver may
    run it: the process launches its two ranks itself (ranks sharing cuda:0
    under XDPGPU_BENCH_REHEARSE=1), and the one rank-0 line reports both
    ranks' frames."""
    import json
    import subprocess
    import sys
    env = dict(os.environ, XDPGPU_BENCH_REHEARSE="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--frames", str(1 << 20),
                        "--steps", "3", "--warmup", "1", "--no-cpu", "--legs", "1500",
                        "--frames-1500", str(1 << 15), "--no-e2e"],
                       capture_output=True, text=True, timeout=240, env=env,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    js = json.loads(lines[0])
    assert js["n_gpus"] == 2 and js["verdicts_ok"] is True and js["value"] > 0
    assert js["config"]["parallelism"] == "shard2"
    assert js["config"]["frames_per_gpu"] == 1 << 20
    # per-rank numbers of the 64 B leg, and the 1500 B leg on every rank
    assert [p["rank"] for p in js["per_rank"]] == [0, 1]
    assert all(p["verdicts_ok"] and p["mpps"] > 0 and p["gpu_span_ms_per_step"] > 0
               for p in js["per_rank"])
    assert len(js["devices"]["pci_bus_ids"]) == 2 and js["devices"]["rccl"]
    l15 = js["secondary_1500B"]
    assert l15["n_gpus"] == 2 and l15["verdicts_ok"] is True and l15["frames"] == 8 << 15
    assert [p["rank"] for p in l15["per_rank"]] == [0, 1]
    assert all(p["verdicts_ok"] and p["mpps"] > 0 for p in l15["per_rank"])
    # all ranks' frames over the slowest rank's time
    slow = max(p["ms_per_launch"] for p in l15["per_rank"])
    assert abs(l15["mpps"] - 2 * (8 << 15) / slow / 1e3) <= 0.1 + 1e-3 * l15["mpps"]
