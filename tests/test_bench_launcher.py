"""bench.py --gpus N: the N ranks are started by bench.py itself (a child
torch.distributed.run, one process per GPU) when it does not already run
under one, and a launch whose rank count differs from --gpus fails loudly
(the driver's scaling run is ``bench.py --gpus N``)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_launch_command_shape():
    cmd = bench.rank_launch_command(8, ["--gpus", "8", "--steps", "5"], 29999)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29999" in cmd
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "5"]


def test_world_must_match_gpus():
    assert bench.check_world(1, {}) == 1
    assert bench.check_world(4, {"WORLD_SIZE": "4"}) == 4
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        bench.check_world(8, {"WORLD_SIZE": "2"})


def test_launched_ranks_see_world(tmp_path):
    """The command bench.py builds really starts N ranks that see WORLD_SIZE=N
    (a stand-in script replaces bench.py: no GPU here)."""
    script = tmp_path / "probe.py"
    script.write_text("import os, sys\nr = os.environ['RANK']\n"
                      "open(os.path.join(sys.argv[1], 'rank' + r), 'w').write(os.environ['WORLD_SIZE'])\n")
    cmd = bench.rank_launch_command(2, [str(tmp_path)], bench.free_port(), script=str(script))
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert sorted(p.name for p in tmp_path.glob("rank*")) == ["rank0", "rank1"]
    assert all(p.read_text() == "2" for p in tmp_path.glob("rank*"))


def test_mismatched_launch_exits_nonzero():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env,
                         capture_output=True, text=True, timeout=120)
    assert out.returncode != 0 and "WORLD_SIZE=2" in out.stderr
