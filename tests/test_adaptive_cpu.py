"""Adaptive FEC controller (adaptive.rs:44-631) through the C ABI without a
GPU (controller-only objects), against the float32 restatement in
oracle/adaptive_ref.py and the reference's own test contracts."""
import sys
from pathlib import Path

import numpy as np
import pytest

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "oracle"))
import adaptive_ref as ref  # noqa: E402

from quicfuscate_amd import _lib as L  # noqa: E402
from quicfuscate_amd import fec  # noqa: E402

M = fec.FecMode


def test_params_ranges_ratios():
    # adaptive.rs:124-153 with the default windows
    assert fec.ModeManager.params_for(M.Light, 16) == (16, 17)
    assert fec.ModeManager.params_for(M.Normal, 64) == (64, 74)
    assert fec.ModeManager.params_for(M.Medium, 128) == (128, 167)
    assert fec.ModeManager.params_for(M.Strong, 512) == (512, 768)
    assert fec.ModeManager.params_for(M.Extreme, 1024) == (1024, 2048)
    assert fec.ModeManager.params_for(M.Zero, 0) == (0, 0)
    for m, rng in zip(M, ref.RANGE):
        assert fec.ModeManager.window_range(m) == rng
        assert np.float32(fec.ModeManager.overhead_ratio(m)) == ref.RATIO[int(m)]
    for m in M:
        for w in list(range(0, 300)) + [511, 512, 1023, 4096]:
            assert fec.ModeManager.params_for(m, w) == ref.params_for(int(m), w), (m, w)


def test_mode_parse_aliases():
    assert fec.FecMode.parse("mittel") == M.Medium and fec.FecMode.parse("5") == M.Extreme
    with pytest.raises(ValueError):
        fec.FecMode.parse("turbo")


@pytest.mark.parametrize("field,value", [("lambda_", 1.5), ("lambda_", -0.1), ("burst_window", 0),
                                         ("hysteresis", 1.0), ("hysteresis", -0.5)])
def test_config_validate_rejects(field, value):
    # adaptive.rs:455-471
    cfg = fec.FecConfig()
    cfg.validate()
    setattr(cfg, field, value)
    with pytest.raises(fec.QfError):
        cfg.validate()
    cfg = fec.FecConfig(kalman_enabled=True, kalman_q=0.0)
    with pytest.raises(fec.QfError):
        cfg.validate()


def _cfg(**kw):
    base = dict(lambda_=0.01, burst_window=50, hysteresis=0.02, pid=fec.PidConfig(1.0, 0.0, 0.0))
    base.update(kw)
    return fec.FecConfig(**base)


def test_extreme_mode_trigger():
    # adaptive.rs:720-740: 18 of 20 lost -> emergency override to Extreme
    a = fec.AdaptiveFec(_cfg(), codec=False, now=0.0)
    a.report_loss(18, 20, now=0.0)
    assert a.current_mode() == M.Extreme
    assert a.is_transitioning()


def test_adaptive_transition_from_toml_values():
    """adaptive.rs:798-816 expects Extreme after report_loss(15, 20) with a
    10-packet burst window, but LossEstimator keeps only the last 10 outcomes
    (5 lost, 5 received: 0.5, adaptive.rs:75-86), which does not exceed
    0.50 + 0.02, and the dwell blocks the PID: the reference stays in Zero.
    Same decision here and in the restatement."""
    a = fec.AdaptiveFec(fec.FecConfig(lambda_=0.1, burst_window=10, pid=fec.PidConfig(1.0, 0.0, 0.0)),
                        codec=False, now=0.0)
    a.report_loss(15, 20, now=0.0)
    c = ref.Controller(lam=0.1, burst=10, kp=1.0, ki=0.0, kd=0.0, now=0.0)
    c.report_loss(15, 20, 0.0)
    assert a.current_mode() == M.Zero and c.mode == ref.ZERO
    assert a.state()["estimated_loss"] == pytest.approx(0.5)
    # one more heavy report pushes the window over the override threshold
    a.report_loss(10, 10, now=0.0)
    assert a.current_mode() == M.Extreme


def test_cross_fade_reference_scenario_has_no_transition():
    """adaptive.rs:742-768 / tests/cross_fade.rs: report_loss(10, 20) right
    after construction.  0.5 does not exceed 0.50 + 0.02 (no override) and the
    500 ms dwell blocks the PID, so the reference does NOT start a cross-fade
    and those tests fail as written; this build decides the same way."""
    a = fec.AdaptiveFec(_cfg(), codec=False, now=0.0)
    a.report_loss(10, 20, now=0.0)
    c = ref.Controller(lam=0.01, burst=50, kp=1.0, ki=0.0, kd=0.0, now=0.0)
    c.report_loss(10, 20, 0.0)
    assert not a.is_transitioning() and c.transition_left == 0
    assert a.current_mode() == M.Zero


def test_cross_fade_countdown():
    # adaptive.rs:537-543: 32 sends end the fade; the old encoder goes at 16
    a = fec.AdaptiveFec(_cfg(initial_mode=M.Normal), codec=False, now=0.0)
    a.report_loss(0, 20, now=1.0)   # PID (sign as written) steps Normal -> Medium
    st = a.state()
    assert st["mode"] == M.Medium and st["transitioning"] and st["transition_left"] == 32
    out = []
    for i in range(32):
        assert a.on_send(fec.Packet(i, bytearray([i] * 8), 8, True), out) == L.QF_OK
        assert a.state()["transition_left"] == 31 - i
    assert not a.is_transitioning()
    assert len(out) == 32 and all(p.is_systematic for p in out)   # no codec objects here


def test_lost_more_than_total_is_einval():
    a = fec.AdaptiveFec(fec.FecConfig(), codec=False, now=0.0)
    with pytest.raises(fec.QfError) as e:
        a.report_loss(5, 3, now=1.0)
    assert e.value.status == L.QF_EINVAL


@pytest.mark.parametrize("seed", range(24))
def test_controller_matches_restatement(seed):
    """Random loss reports and clock readings: every decision (mode, window,
    k, n, fade countdown) and the f32 loss estimate equal the restatement's."""
    rng = np.random.default_rng(seed)
    kalman = bool(rng.integers(0, 2))
    lam = float(np.float32(rng.uniform(0.01, 0.9)))
    burst = int(rng.integers(1, 60))
    hyst = float(np.float32(rng.uniform(0.0, 0.2)))
    kp, ki, kd = (float(np.float32(x)) for x in rng.uniform(-0.5, 2.0, 3))
    initial = int(rng.integers(0, 6))
    q, r = float(np.float32(rng.uniform(1e-4, 0.01))), float(np.float32(rng.uniform(1e-3, 0.1)))
    t = float(rng.integers(0, 4)) * 0.25
    cfg = fec.FecConfig(lambda_=lam, burst_window=burst, hysteresis=hyst, pid=fec.PidConfig(kp, ki, kd),
                        initial_mode=M(initial), kalman_enabled=kalman, kalman_q=q, kalman_r=r)
    a = fec.AdaptiveFec(cfg, codec=False, now=t)
    c = ref.Controller(lam, burst, hyst, kp, ki, kd, initial, (q, r) if kalman else None, now=t)
    for step in range(60):
        t += float(rng.choice([0.0, 0.125, 0.25, 0.5, 0.75, 2.0]))
        total = int(rng.integers(0, 40))
        lost = int(rng.integers(0, total + 1)) if total else 0
        if rng.random() < 0.15:       # burst of heavy loss
            lost = total
        a.report_loss(lost, total, now=t)
        c.report_loss(lost, total, t)
        for _ in range(int(rng.integers(0, 20))):
            a.on_send(fec.Packet(step, bytearray(4), 4, True), [])
            c.on_send()
        s, w = a.state(), c.state()
        assert (int(s["mode"]), s["window"], s["k"], s["n"], s["transition_left"]) == \
            (w["mode"], w["window"], w["k"], w["n"], w["transition_left"]), (seed, step)
        assert np.float32(s["estimated_loss"]) == np.float32(w["estimated_loss"]), (seed, step)
