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


def test_n_gt_1_value_is_the_gathered_step():
    """At N > 1 ``value`` is north_star's step (shard + all-reduce + the RCCL
    all-gather of the marginal tensor) and the rank-local step is reported
    beside it; --rank-local swaps them; N = 1 is the fused single launch."""
    m = bench.step_modes(bench.parse(["--gpus", "2"]), 2)
    assert m["sharded"] and m["gather"] and m["value_kind"] == "gathered"
    assert "all-gather" in m["parallelism"] and m["other_kind"] == "rank_local"
    assert not m["fold"]  # fold ring with real peers: off until pinned on >= 2 GPUs
    m = bench.step_modes(bench.parse(["--gpus", "2", "--rank-local"]), 2)
    assert not m["gather"] and m["value_kind"] == "rank_local" and m["other_kind"] == "gathered"
    assert "no all-gather" in m["parallelism"]
    m = bench.step_modes(bench.parse([]), 1)
    assert not m["sharded"] and m["value_kind"] == "single_process" and m["other_kind"] is None
    m = bench.step_modes(bench.parse(["--sharded"]), 1)
    assert m["sharded"] and not m["gather"] and m["fold"]
    p = bench.projection(8)
    assert p["gathered_x_vs_1gpu"] < 2.0 < p["rank_local_x_vs_1gpu"]
    # the communicator's rank count must equal --gpus
    assert bench.multi_gpu_fields(2, 2, 2)["rccl_ranks"] == 2
    assert bench.multi_gpu_fields(1, 1, None) == {"rccl_ranks": None}
    with pytest.raises(SystemExit, match="communicator has 1 ranks"):
        bench.multi_gpu_fields(2, 2, 1)


STANDIN_MODES = """
import json, os, sys
sys.path.insert(0, {root!r})
import bench
world = bench.check_world(2, os.environ)
m = bench.step_modes(bench.parse(["--gpus", "2"]), world)
line = {{"n_gpus": world, "value_kind": m["value_kind"], "config": {{"parallelism": m["parallelism"]}}}}
line["value_" + m["other_kind"]] = 1.0
# the stepper's RCCL communicator is stood in for by the gloo group's size
import torch.distributed as dist
dist.init_process_group("gloo")
line.update(bench.multi_gpu_fields(2, world, dist.get_world_size()))
dist.destroy_process_group()
open(os.path.join(sys.argv[1], "line" + os.environ["RANK"]), "w").write(json.dumps(line))
"""


def test_two_rank_launch_line_names_the_all_gather(tmp_path):
    """Through the 2-rank launch bench.py uses: each rank's line names the
    all-gather in ``parallelism`` and carries ``value_rank_local``."""
    import json

    script = tmp_path / "modes.py"
    script.write_text(STANDIN_MODES.format(root=ROOT))
    cmd = bench.rank_launch_command(2, [str(tmp_path)], bench.free_port(), script=str(script))
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    for r in (0, 1):
        line = json.loads((tmp_path / f"line{r}").read_text())
        assert line["n_gpus"] == 2 and line["value_kind"] == "gathered"
        assert "all-gather" in line["config"]["parallelism"] and "value_rank_local" in line
        assert line["rccl_ranks"] == 2
        p = line["projection"]
        assert p["link_assumption"].startswith("assumed") and "not a measurement" in p["status"]
        assert p["gathered_x_vs_1gpu_if_bidirectional"] <= p["gathered_x_vs_1gpu"]


STANDIN_STALL = """
import os, sys, time
sys.path.insert(0, {root!r})
import torch, torch.distributed as dist
from continuousbayesiannetwork_amd.distributed import Watchdog
dist.init_process_group("gloo")
rank = dist.get_rank()
wd = Watchdog({bound}, what="(stand-in N>1 bench)")
wd.arm(phase="timed region")
x = torch.zeros(1)
for i in range(1, 1000):
    if rank == 1 and i > 3:
        wd.disarm()  # rank 1 stops issuing steps (busy elsewhere, not stuck: only rank 0 must report)
        time.sleep(600)
    wd.beat(step=i, op="all_reduce(max) of the block max words")
    dist.all_reduce(x, op=dist.ReduceOp.MAX)
print("unreachable", flush=True)
"""


def test_watchdog_ends_a_stalled_two_rank_run(tmp_path):
    """Rank 1 stops issuing steps: rank 0, blocked in the step's collective,
    reports its step index / last collective within the bound and exits
    non-zero; torch.distributed.run stops rank 1 and bench.launch_ranks
    returns the failure."""
    import time

    script = tmp_path / "stall.py"
    script.write_text(STANDIN_STALL.format(root=ROOT, bound=3.0))
    a = bench.parse(["--gpus", "2"])
    log = tmp_path / "err.txt"
    t0 = time.monotonic()
    with open(log, "w") as fh:
        import contextlib

        with contextlib.redirect_stderr(fh):
            # launch_ranks inherits this process's fds: capture at the fd level
            rc = subprocess.run([sys.executable, "-c",
                                 "import sys; sys.path.insert(0, %r); import bench; "
                                 "sys.exit(bench.launch_ranks(bench.parse(['--gpus', '2']), [], script=%r))"
                                 % (ROOT, str(script))],
                                stdout=fh, stderr=subprocess.STDOUT, timeout=180).returncode
    dt = time.monotonic() - t0
    err = log.read_text()
    assert a.gpus == 2
    assert rc != 0, err
    assert "[cbn watchdog] rank 0/2" in err and "step=4" in err and "all_reduce" in err, err
    assert "unreachable" not in err
    assert dt < 120, dt
