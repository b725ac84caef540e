#!/usr/bin/env python3
"""The reference's benches/fec_modes.rs on the MI355X: AdaptiveFec::on_send of
a 1,024-byte packet per mode (Light, Normal, Medium, Strong, and Extreme,
which the reference bench leaves out), the window full, so every call
slides the window and emits the n - k repairs (adaptive.rs:519-562).
Reports microseconds per on_send and repair payload bytes per second, beside
the oracle's single-thread encode of the same window (the work of one call).

    python tools/bench_fec_modes.py [--calls 200] [--out gpurun_out/fec_modes.json]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def main():
    from quicfuscate_amd import _lib as L
    from quicfuscate_amd import fec as qf
    from tests import oracle_py as oracle

    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("--len", type=int, default=1024)
    ap.add_argument("--out", default="gpurun_out/fec_modes.json")
    a = ap.parse_args()
    M = qf.FecMode
    res = {}
    payload = bytearray([0xAB] * a.len)   # fec_modes.rs:9-12
    for mode in (M.Light, M.Normal, M.Medium, M.Strong, M.Extreme):
        fec = qf.AdaptiveFec(qf.FecConfig(initial_mode=mode, max_len=2048), now=0.0)
        st = fec.state()
        k, n = st["k"], st["n"]
        q = []
        # fill the window (the reference bench reaches steady state the same way)
        t0 = time.perf_counter()
        for i in range(k):
            s = fec.on_send(qf.Packet(i, bytearray(payload), a.len, True), q)
            q.clear()
        fill_s = time.perf_counter() - t0
        calls = a.calls if mode != M.Extreme else max(10, a.calls // 10)
        t0 = time.perf_counter()
        for i in range(calls):
            s = fec.on_send(qf.Packet(k + i, bytearray(payload), a.len, True), q)
            emitted = len(q)
            q.clear()
        dt = (time.perf_counter() - t0) / calls
        r = n - k
        entry = {"k": k, "n": n, "status": int(s), "packets_per_call": emitted, "us_per_on_send": round(dt * 1e6, 1),
                 "window_fill_s": round(fill_s, 3)}
        if s == L.QF_OK and r:
            entry["repair_MiBps"] = round(r * a.len / dt / 2**20, 1)
            # the work of one call on the CPU: the window's r repairs (oracle, 1 thread)
            src = np.full((k, a.len), 0xAB, np.uint8)
            t0 = time.perf_counter()
            if mode == M.Extreme:
                rr = 16
                oracle.encode16(src, rr)
                cpu = (time.perf_counter() - t0) * r / rr
            else:
                oracle.encode(src, r)
                cpu = time.perf_counter() - t0
            entry["oracle_us_per_call"] = round(cpu * 1e6, 1)
        res[mode.name] = entry
        print(mode.name, entry, flush=True)
        fec.close()
    Path(a.out).parent.mkdir(exist_ok=True)
    Path(a.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
