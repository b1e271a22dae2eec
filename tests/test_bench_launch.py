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
