"""Rehearsal of the driver's multi-GPU bench launch on one GPU: two ranks
under torch.distributed.run (gloo, both ranks on cuda:0) must finish, verify
their decodes, and report distinct per-rank repair folds (each rank encodes
its own generations: weak scaling, no data-path collective)."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
REPO = Path(__file__).resolve().parent.parent


def _run(cmd, env, tmp_path, timeout=170):
    """Run bench.py; returns (compact stdout line, full detail record)."""
    detail = tmp_path / "detail.json"
    p = subprocess.run(cmd + ["--detail", str(detail)], cwd=REPO, env=env, capture_output=True, text=True,
                       timeout=timeout)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith('{"metric"')]
    assert len(lines) == 1, p.stdout[-2000:]   # rank 0 prints exactly one line
    import bench  # noqa: F401  (LINE_MAX)
    assert len(lines[0]) <= bench.LINE_MAX, len(lines[0])
    return json.loads(lines[0]), json.loads(detail.read_text())


def test_bench_two_ranks_gloo_rehearsal(tmp_path):
    env = dict(os.environ, QF_BENCH_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29531", str(REPO / "bench.py"), "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--G", "2048", "--c4-G", "3000", "--c4-steps", "2", "--rank-sample", "8"]
    line, d = _run(cmd, env, tmp_path)
    assert line["n_gpus"] == 2 and line["verified"] and line["process_group"]["backend"] == "gloo"
    assert line["descriptor_matches_by_rank"] == [True, True] and line["c4"]["verified"]
    assert d["n_gpus"] == 2 and d["verified"] and d["scaling"] == "weak"
    folds = d["repair_xor_fold_by_rank"]
    assert len(folds) == 2 and folds[0] != folds[1]
    assert d["value"] > 0 and d["ms_per_step"] > 0
    # the headline is the same per-GPU workload at every N (C2 + C3 shape);
    # the C4 leg (reduced G here) has its own timing, verification and
    # per-rank oracle samples; the process group's own world size, and the
    # sliding-window halo leg over it
    assert d["config"]["workload"].startswith("C2") and d["config"]["generations_per_gpu"] == 2048
    c4 = d["c4"]
    assert c4["ranks"] == 2 and c4["generations_per_rank"] == 3000 and c4["verified"]
    assert c4["value"] > 0 and c4["oracle_sample_generations_per_rank"] == 8
    assert d["process_group"]["world_size"] == 2 and d["process_group"]["backend"] == "gloo"
    assert d["run_descriptor"]["broadcast_from_rank0"] and d["run_descriptor"]["matches_by_rank"] == [True, True]
    sh = d["sliding_halo"]
    assert sh["first_window_matches"] and sh["halo_packets"] == 63 and sh["ms_per_step_max"] > 0


def test_bench_gpus_without_launcher_spawns_ranks(tmp_path):
    """`bench.py --gpus 2` with no WORLD_SIZE in the environment starts its two
    ranks itself (torch.distributed.run as a child, before any GPU call) and
    reports n_gpus == 2 -- never a 1-GPU line for --gpus 2.  (gloo: both ranks
    share cuda:0 on this box.)"""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(QF_BENCH_BACKEND="gloo", MASTER_PORT="29533")
    cmd = [sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1", "--G", "1024",
           "--c4-G", "0", "--no-cpu", "--host-path-G", "0", "--c3b-G", "0", "--c5-mixed-bytes", "0"]
    d, _ = _run(cmd, env, tmp_path)
    assert d["n_gpus"] == 2 and d["process_group"]["world_size"] == 2 and d["verified"]


def test_bench_c4_full_size_leg_one_gpu(tmp_path):
    """The C4 leg at its real size on one GPU: 156,250 generations = 10 M
    packets, encode + decode (12.6 GB of received rows), every recovered byte
    checked on the device, 16 seeded generations against the CPU oracle."""
    cmd = [sys.executable, str(REPO / "bench.py"), "--steps", "2", "--warmup", "1", "--G", "1024",
           "--c4-G", "156250", "--c4-steps", "2", "--rank-sample", "16", "--no-cpu", "--host-path-G", "0",
           "--c3b-G", "0", "--c5-mixed-bytes", "0"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    line, d = _run(cmd, env, tmp_path)
    assert line["c4"]["verified"] and line["c4"]["generations_per_rank"] == 156250
    c4 = d["c4"]
    assert c4["generations_per_rank"] == 156250 and c4["packets_per_rank"] == 10_000_000
    assert c4["verified"] and c4["value"] > 0


def test_bench_c5_leg_small(tmp_path):
    """The line's c5 leg (BASELINE configs[4]) at reduced bytes: the
    heterogeneous batch round-trips, every shape's block decode and sliding
    windows verify on the device, and no byte accounting exceeds the HBM roof
    (sliding windows priced at (1 + r) L)."""
    cmd = [sys.executable, str(REPO / "bench.py"), "--steps", "2", "--warmup", "1", "--G", "1024", "--c4-G", "0",
           "--no-cpu", "--host-path-G", "0", "--c3b-G", "0", "--c5-mixed-bytes", "2e8", "--c5-shape-bytes", "5e7"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    line, d = _run(cmd, env, tmp_path)
    lc5 = line["c5"]
    assert lc5["verified"] and lc5["mixed"]["round_trip_ok"] and len(lc5["shapes"]) == 7
    for leg in ("encode", "decode"):
        m = lc5["mixed"][leg]
        # device span of the call (HIP events) against the sum of its kernels
        assert m["span_gibps"] > 0 and m["kernel_gibps"] > 0 and m["span_over_kernel"] > 0.9, m
    c5 = d["c5"]
    assert c5["mixed_desc_batch"]["round_trip_ok"]
    shapes = [key for key in c5 if key.startswith("k")]
    assert len(shapes) == 7
    for key in shapes:
        s = c5[key]
        assert s["block/decode"]["verified"] and s["sliding/encode"]["verified"], key
        for mode in ("block/encode", "sliding/encode", "block/decode"):
            assert 0 < s[mode]["hbm_frac_of_8TBps"] < 1.0, (key, mode, s[mode]["hbm_frac_of_8TBps"])
        assert s["sliding/encode"]["bytes_rule"].startswith("(1 + r) L")
        v = s["sliding/encode"]["valu"]
        assert v is None or 0 < v["frac"] <= 1.05, (key, v)


def test_bench_rccl_branch_one_rank(tmp_path):
    """VERDICT r04 missing 2: the nccl (RCCL) branch the 8-GPU driver run takes,
    executed once at world size 1 -- init_process_group("nccl", device_id=...),
    the device-tensor broadcast of the run descriptor, the all_gather of the
    repair folds and flags, the MAX all_reduce of the step times, barriers,
    and the sliding-window leg's collectives."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "QF_BENCH_BACKEND")}
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", "29537", str(REPO / "bench.py"), "--gpus", "1",
           "--force-pg", "--steps", "2", "--warmup", "1", "--G", "2048", "--c4-G", "3000", "--c4-steps", "2",
           "--rank-sample", "8", "--no-cpu", "--host-path-G", "0", "--c3b-G", "0", "--c5-mixed-bytes", "0"]
    line, d = _run(cmd, env, tmp_path)
    assert line["process_group"] == {"backend": "nccl", "world_size": 1, "env_world_size": 1}
    assert line["verified"] and line["descriptor_matches_by_rank"] == [True]
    assert len(line["repair_xor_fold_by_rank"]) == 1 and line["c4"]["verified"]
    assert d["run_descriptor"]["broadcast_from_rank0"]
    sh = d["sliding_halo"]
    assert sh["backend"] == "nccl" and sh["first_window_matches"] and sh["ms_per_step_max"] > 0
