# SPDX-License-Identifier: GPL-2.0
"""bench.py --gpus N as its own launcher (CPU): the plan (rank or launcher)
from --gpus and the environment, the ranks' environments, and the
launcher's handling of its children (all finish; one fails and the others
are stopped).  The GPU form is tests/test_shard.py::test_bench_self_launch."""
import os
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_world_plan():
    assert bench.world_plan(1, {}, 1, False) == "run"
    assert bench.world_plan(8, {}, 8, False) == "launch"
    assert bench.world_plan(8, {"WORLD_SIZE": "8"}, 8, False) == "run"
    # ranks sharing GPUs only when rehearsing
    assert bench.world_plan(2, {}, 1, True) == "launch"
    with pytest.raises(SystemExit):
        bench.world_plan(2, {}, 1, False)
    with pytest.raises(SystemExit):
        bench.world_plan(1, {}, 0, False)
    # an outer launcher and --gpus disagreeing is an error, not a silent N
    with pytest.raises(SystemExit):
        bench.world_plan(8, {"WORLD_SIZE": "2"}, 8, False)
    with pytest.raises(SystemExit):
        bench.world_plan(0, {}, 8, False)


def test_rank_envs():
    envs = bench.rank_envs(4, {"X": "1"}, 12345)
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    for e in envs:
        assert e["WORLD_SIZE"] == "4" and e["MASTER_ADDR"] == "127.0.0.1"
        assert e["MASTER_PORT"] == "12345" and e["X"] == "1"
        assert e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_launch_ranks_all_finish(tmp_path):
    code = ("import os, sys; open(os.path.join(sys.argv[1], os.environ['RANK']), 'w')"
            ".write(os.environ['LOCAL_RANK'] + ' ' + os.environ['WORLD_SIZE'])")
    rc = bench.launch_ranks([sys.executable, "-c", code, str(tmp_path)], 3)
    assert rc == 0
    got = {p.name: p.read_text() for p in tmp_path.iterdir()}
    assert got == {"0": "0 3", "1": "1 3", "2": "2 3"}


def test_launch_ranks_failure_stops_the_rest(tmp_path):
    # rank 1 fails at once; rank 0 would sleep a minute (a rank stuck in a
    # collective): the launcher returns rank 1's code and stops rank 0
    code = ("import os, sys, time\n"
            "if os.environ['RANK'] == '1': sys.exit(3)\n"
            "time.sleep(60)\n"
            "open(os.path.join(sys.argv[1], 'done'), 'w').write('x')\n")
    t0 = time.time()
    rc = bench.launch_ranks([sys.executable, "-c", code, str(tmp_path)], 2)
    assert rc == 3
    assert time.time() - t0 < 30
    assert not (tmp_path / "done").exists()


def test_gather_leg_child(monkeypatch):
    """The gather leg runs in a child process (tools/e2e_probe.py): its last
    JSON line becomes the leg, a failing or hung child becomes an error
    entry, and the bench's line survives either way."""
    import json
    import subprocess
    ceil = {"h2d_gbps": 57.0, "d2h_gbps": 56.0}
    seen = {}

    def ok(cmd, **kw):
        seen["cmd"] = cmd
        line = json.dumps({"mpps": 250.0, "mode": "gather", "verdicts_ok": True})
        return subprocess.CompletedProcess(cmd, 0, "log line\n" + line + "\n", "")
    monkeypatch.setattr(bench.subprocess, "run", ok)
    r = bench.gather_leg(1 << 20, 32, ceil)
    assert r["mpps"] == 250.0 and "mode" not in r and r["pcie_ceiling"] == ceil
    cmd = seen["cmd"]
    assert cmd[1].endswith(os.path.join("tools", "e2e_probe.py"))
    assert "--gather-only" in cmd and cmd[cmd.index("--frames") + 1] == str(1 << 20)
    assert cmd[cmd.index("--h2d-ceil") + 1] == "57.0"

    def fault(cmd, **kw):
        return subprocess.CompletedProcess(cmd, -6, "", "illegal memory access\n")
    monkeypatch.setattr(bench.subprocess, "run", fault)
    r = bench.gather_leg(1 << 20, 32, ceil)
    assert "error" in r and "-6" in r["error"] and "illegal" in r["error"]

    def hang(cmd, **kw):
        raise subprocess.TimeoutExpired(cmd, kw.get("timeout"))
    monkeypatch.setattr(bench.subprocess, "run", hang)
    assert "timed out" in bench.gather_leg(1 << 20, 32, ceil)["error"]


def test_check_distinct_devices():
    """One rank per GPU unless rehearsing: two ranks on one device (same
    UUID and same PCI bus id) is an error naming both ranks; one UUID, or
    one bus id, reported for distinct devices is not."""
    a = {"pci_bus_id": "0000:05:00", "uuid": "u0"}
    b = {"pci_bus_id": "0000:15:00", "uuid": "u1"}
    bench.check_distinct_devices([a, b], False)
    with pytest.raises(SystemExit, match="ranks 0 and 1 share"):
        bench.check_distinct_devices([a, dict(a)], False)
    with pytest.raises(SystemExit, match="ranks 1 and 2 share"):
        bench.check_distinct_devices([a, dict(b, uuid=""), dict(b, uuid="")], False)
    bench.check_distinct_devices([a, dict(a)], True)
    bench.check_distinct_devices([a, dict(b, uuid="u0")], False)
    bench.check_distinct_devices([a, dict(b, pci_bus_id=a["pci_bus_id"])], False)


def _gather_rank(rank, world, port, out_dir):
    import json
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world,
                            timeout=__import__("datetime").timedelta(seconds=60))
    got = bench.gather_ranks({"rank": rank, "ms": 1.0 + rank}, world)
    ident = {"pci_bus_id": f"0000:{rank:02x}:00", "uuid": f"u{rank}"}
    idents = bench.gather_ranks(ident, world)
    bench.check_distinct_devices(idents, False)
    if rank == 0:
        with open(os.path.join(out_dir, "got.json"), "w") as f:
            json.dump({"got": got, "idents": idents}, f)
    dist.barrier()
    dist.destroy_process_group()


def test_gather_ranks_gloo(tmp_path):
    """The per-rank list of the N-rank line (bench.gather_ranks over gloo,
    two processes): every rank's dict in rank order, and the distinct-device
    check over the gathered identities."""
    import json
    import torch.multiprocessing as mp
    mp.spawn(_gather_rank, args=(2, bench.free_port(), str(tmp_path)), nprocs=2, join=True)
    js = json.loads((tmp_path / "got.json").read_text())
    assert js["got"] == [{"rank": 0, "ms": 1.0}, {"rank": 1, "ms": 2.0}]
    assert [d["uuid"] for d in js["idents"]] == ["u0", "u1"]
    assert bench.gather_ranks({"rank": 0}, 1) == [{"rank": 0}]
