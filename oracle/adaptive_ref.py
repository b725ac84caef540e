"""CPU restatement of the reference's adaptive FEC controller -- TEST
INFRASTRUCTURE ONLY (imported by tests/, never by the library).

Follows /root/reference/src/fec/adaptive.rs and mod.rs line by line with
numpy float32 scalars, so every f32 operation rounds as Rust's does:
  LossEstimator        adaptive.rs:44-99
  KalmanFilter         mod.rs:56-79
  ModeManager          adaptive.rs:102-279 (thresholds 161-166, dwell 181,
                       window_range 124-133, overhead_ratio 135-147,
                       params_for 149-153, update 189-258)
  PidController        adaptive.rs:282-324
  AdaptiveFec          adaptive.rs:326-631 (codec state only: configuration,
                       cross-fade countdown; payload coding is checked by the
                       codec's own parity tests)
Time is injected (seconds, float) instead of Instant::now().
Parity note: the reference crate cannot be built here (no Rust toolchain,
SURVEY F1), so this restatement is pinned by the reference's test contracts
that its semantics can meet (extreme_mode_trigger, parse_config/validate,
params_for values) -- its cross-fade tests cannot pass as written
(DESIGN.md section 7).
"""
from __future__ import annotations

from collections import deque

import numpy as np

F = np.float32
ZERO, LIGHT, NORMAL, MEDIUM, STRONG, EXTREME = range(6)
THRESH = [F(0.01), F(0.05), F(0.15), F(0.30), F(0.50), F(1.0)]
RATIO = [F(1.0), F(1.05), F(1.15), F(1.30), F(1.50), F(2.0)]
RANGE = [(0, 0), (8, 32), (32, 128), (64, 256), (256, 1024), (1024, 4096)]
DEFAULT_WINDOWS = [0, 16, 64, 128, 512, 1024]
CROSS_FADE_LEN = 32
MIN_DWELL = F(0.5)
ALPHA_K = F(0.5)


def sat_usize(x) -> int:
    """Rust `f32 as usize` (saturating; NaN -> 0)."""
    x = float(x)
    if not x > 0.0:
        return 0
    return int(x)


def round_half_away(x):
    """f32::round."""
    x = F(x)
    r = np.floor(np.abs(x) + F(0.5))
    return F(np.copysign(r, x))


def params_for(mode: int, window: int):
    return window, sat_usize(np.ceil(F(window) * RATIO[mode]))


class Kalman:
    def __init__(self, q, r):
        self.estimate, self.error_cov, self.q, self.r = F(0.0), F(1.0), F(q), F(r)

    def update(self, m):
        self.error_cov = F(self.error_cov + self.q)
        k = F(self.error_cov / F(self.error_cov + self.r))
        self.estimate = F(self.estimate + F(k * F(F(m) - self.estimate)))
        self.error_cov = F(self.error_cov * F(F(1.0) - k))
        return self.estimate


class LossEstimator:
    def __init__(self, lam, cap, kalman=None):
        self.ema, self.lam, self.cap, self.kf = F(0.0), F(lam), cap, kalman
        self.win = deque()

    def report(self, lost, total):
        cur = F(F(lost) / F(total)) if total > 0 else F(0.0)
        if self.kf is not None:
            cur = self.kf.update(cur)
        self.ema = F(F(self.lam * cur) + F(F(F(1.0) - self.lam) * self.ema))
        for v in [True] * lost + [False] * (total - lost):
            if len(self.win) == self.cap:
                self.win.popleft()
            self.win.append(v)

    def estimate(self):
        burst = F(0.0) if not self.win else F(F(sum(self.win)) / F(len(self.win)))
        return max(self.ema, burst)


class Pid:
    def __init__(self, kp, ki, kd, now):
        self.kp, self.ki, self.kd = F(kp), F(ki), F(kd)
        self.integral, self.prev = F(0.0), F(0.0)
        self.last = now

    def update(self, cur, setpoint, now):
        dt = F(max(0.0, now - self.last))
        self.last = now
        if not dt > 0:
            return F(0.0)
        err = F(F(setpoint) - F(cur))
        self.integral = F(self.integral + F(err * dt))
        der = F(F(err - self.prev) / dt)
        self.prev = err
        return F(F(F(self.kp * err) + F(self.ki * self.integral)) + F(self.kd * der))


class Controller:
    """AdaptiveFec's configuration state."""

    def __init__(self, lam=0.1, burst=20, hyst=0.02, kp=1.2, ki=0.5, kd=0.1, initial=ZERO, kalman=None,
                 windows=None, now=0.0):
        self.windows = list(windows or DEFAULT_WINDOWS)
        self.est = LossEstimator(lam, burst, Kalman(*kalman) if kalman else None)
        self.mode = initial
        self.window = self.windows[initial]
        self.last_change = now
        self.hyst = F(hyst)
        self.pid = Pid(kp, ki, kd, now)
        self.k, self.n = params_for(self.mode, self.window)
        self.transition_left = 0

    def _update(self, est, now):
        if est > F(THRESH[STRONG] + self.hyst):
            prev = (self.mode, self.window)
            self.mode = EXTREME
            self.window = self.windows[EXTREME]
            self.last_change = now
            return prev
        if F(max(0.0, now - self.last_change)) < MIN_DWELL:
            return None
        out = self.pid.update(est, THRESH[self.mode], now)
        new = self.mode
        if out > F(0.1):
            new = min(self.mode + 1, EXTREME)
        elif out < F(-0.1):
            new = max(self.mode - 1, ZERO) if self.mode > LIGHT else ZERO
        pm, pw = self.mode, self.window
        if new != self.mode:
            self.mode, self.last_change, self.window = new, now, self.windows[new]
        alpha = F(F(1.0) + F(ALPHA_K * F(est - THRESH[self.mode])))
        nw = sat_usize(round_half_away(F(F(self.window) * alpha)))
        lo, hi = RANGE[self.mode]
        self.window = min(max(nw, lo), hi)
        if pm != self.mode or pw != self.window:
            return (pm, pw)
        return None

    def report_loss(self, lost, total, now):
        self.est.report(lost, total)
        prev = self._update(self.est.estimate(), now)
        self.k, self.n = params_for(self.mode, self.window)
        if prev is not None:
            self.transition_left = CROSS_FADE_LEN

    def on_send(self):
        if self.transition_left > 0:
            self.transition_left -= 1

    def state(self):
        return {"mode": self.mode, "window": self.window, "k": self.k, "n": self.n,
                "transition_left": self.transition_left, "estimated_loss": float(self.est.estimate())}
