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


def test_bench_two_ranks_gloo_rehearsal():
    env = dict(os.environ, QF_BENCH_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29531", str(REPO / "bench.py"), "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--G", "2048"]
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=170)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith('{"metric"')]
    assert len(lines) == 1, p.stdout[-2000:]   # rank 0 prints exactly one line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["verified"] and d["scaling"] == "weak"
    folds = d["repair_xor_fold_by_rank"]
    assert len(folds) == 2 and folds[0] != folds[1]
    assert d["value"] > 0 and d["ms_per_step"] > 0
    # C4 shape at N > 1 (reduced G here): per-rank oracle samples, the process
    # group's own world size, and the sliding-window halo leg over it
    assert d["config"]["workload"].startswith("C4") and d["config"]["generations_per_gpu"] == 2048
    assert d["rank_oracle_sample"]["pass_by_rank"] == [True, True]
    assert d["rank_oracle_sample"]["generations_per_rank"] >= 64
    assert d["process_group"]["world_size"] == 2 and d["process_group"]["backend"] == "gloo"
    assert d["run_descriptor"]["broadcast_from_rank0"] and d["run_descriptor"]["matches_by_rank"] == [True, True]
    sh = d["sliding_halo"]
    assert sh["first_window_matches"] and sh["halo_packets"] == 63 and sh["ms_per_step_max"] > 0
