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


def _recorded_full(name="r04am_bench_full.json"):
    import json
    lines = [l for l in (REPO / "profiles" / name).read_text().splitlines() if l.startswith("{")]
    return json.loads(lines[-1])


def test_line_fits_driver_parse():
    """the 20.8 KB round-4 line was not parsed by the
    driver.  The compact line of a recorded full run (every leg present) must
    stay under LINE_MAX and carry the contract keys first."""
    import json
    full = _recorded_full()
    line = bench.compact_line(full, "gpurun_out/bench_detail.json")
    s = json.dumps(line)
    assert len(s) <= bench.LINE_MAX <= 8000, len(s)
    keys = list(line)
    assert keys[:13] == ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                         "scaling", "vs_baseline", "dtype", "data", "config"]
    for k in ("roofline", "cpu_baseline", "roofline_encode", "c5", "c4", "cpu_variants_gibps"):
        assert line.get(k), k
    rl = line["roofline"]
    assert rl["bound"] == "hbm" and rl["unit"] == "GB/s" and 0 < rl["frac"] < 1
    assert abs(rl["achieved"] / rl["peak"] - rl["frac"]) < 1e-3
    cb = line["cpu_baseline"]
    assert cb["kind"] in ("port", "reference") and cb["cores"] >= 1 and cb["value"] > 0
    assert len(line["c5"]["shapes"]) == 7
    assert json.loads(s) == line


def test_line_trims_oversized_legs():
    """Whatever a leg grows into, the line keeps the contract keys and fits."""
    import json
    full = _recorded_full()
    full["cpu_gf_mul_loop"] = {f"k{i}": {"mb_s": i} for i in range(2000)}
    full["cpu_gf_mul_loop"].update({"table": {"mb_s": 1.0}})
    full["c5"]["k32_r5"]["block/encode"]["GiBps_alg"] = "x" * 9000
    line = bench.compact_line(full)
    assert len(json.dumps(line)) <= bench.LINE_MAX
    assert line["roofline"] and line["cpu_baseline"] and line["value"] == full["value"]


def test_detail_written(tmp_path):
    import json
    full = _recorded_full()
    p = bench.emit_detail(full, str(tmp_path / "d.json"))
    assert p and json.loads(open(p).read())["value"] == full["value"]
    assert bench.emit_detail(full, "") is None


def test_cgroup_cpu_quota(tmp_path):
    """The usable-CPU count of cpu_baseline: cgroup v2 cpu.max, else v1 cfs
    quota / period, floored; None without a quota."""
    assert bench.cgroup_cpu_quota(str(tmp_path)) is None
    (tmp_path / "cpu.max").write_text("1600000 100000\n")
    assert bench.cgroup_cpu_quota(str(tmp_path)) == 16
    (tmp_path / "cpu.max").write_text("max 100000\n")
    assert bench.cgroup_cpu_quota(str(tmp_path)) is None
    (tmp_path / "cpu.max").unlink()
    (tmp_path / "cpu").mkdir()
    (tmp_path / "cpu" / "cpu.cfs_quota_us").write_text("250000")
    (tmp_path / "cpu" / "cpu.cfs_period_us").write_text("100000")
    assert bench.cgroup_cpu_quota(str(tmp_path)) == 2
    (tmp_path / "cpu" / "cpu.cfs_quota_us").write_text("-1")
    assert bench.cgroup_cpu_quota(str(tmp_path)) is None
