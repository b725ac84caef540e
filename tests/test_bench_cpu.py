"""bench.py host logic on CPU: the multi-GPU launch decision (no GPU calls)."""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
import bench  # noqa: E402


def _args(**kw):
    a = bench.parse([])
    for k_, v in kw.items():
        setattr(a, k_, v)
    return a


def test_gpus_without_launcher_spawns_ranks():
    plan = bench.launch_plan(_args(gpus=4), {}, ["--gpus", "4", "--steps", "3"])
    assert isinstance(plan, list)
    assert plan[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in plan and "--master-addr=127.0.0.1" in plan
    assert plan[-3:] == ["--gpus", "4", "--steps", "3"] or plan[-4:-1] == ["--gpus", "4", "--steps"]


def test_launcher_world_size_must_match_gpus():
    assert bench.launch_plan(_args(gpus=2), {"WORLD_SIZE": "2"}) is None
    err = bench.launch_plan(_args(gpus=8), {"WORLD_SIZE": "1"})
    assert isinstance(err, str) and "--gpus 8" in err
    # the driver's N=1 run: no launcher, no spawn
    assert bench.launch_plan(_args(gpus=1), {}) is None


def test_main_refuses_mismatched_world_size(monkeypatch):
    """A launcher with WORLD_SIZE=1 and --gpus 8: exit code 2 before any GPU call."""
    monkeypatch.setenv("WORLD_SIZE", "1")
    assert bench.main(["--gpus", "8"]) == 2


def test_headline_workload_is_per_gpu_constant():
    """Every N runs the same generations per GPU (weak scaling); C4 is its own leg."""
    a = bench.parse([])
    assert a.G is None and a.config == "auto" and a.c4_G == 156250
