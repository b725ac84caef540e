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
        # receive side: a fresh generation of packets 0..k-1 with 20 % of the
        # sources lost, completed by the window's repairs (adaptive.rs:566-599)
        if s == L.QF_OK and r:
            snd = qf.AdaptiveFec(qf.FecConfig(initial_mode=mode, max_len=2048), now=0.0)
            rcv = qf.AdaptiveFec(qf.FecConfig(initial_mode=mode, max_len=2048), now=0.0)
            pk = [qf.Packet(i, bytearray(np.random.default_rng(i).integers(0, 256, a.len, dtype=np.uint8).tobytes()),
                            a.len, True) for i in range(k)]
            reps = []
            for p in pk:
                q = []
                snd.on_send(p, q)
                reps = q[1:]
            lost = set(range(0, k, 5)) if r >= len(range(0, k, 5)) else set(range(r))
            # warm-up generation on a separate receiver (first-use allocations)
            warm = qf.AdaptiveFec(qf.FecConfig(initial_mode=mode, max_len=2048), now=0.0)
            for p in [p for p in pk if p.id not in lost] + reps[: len(lost)]:
                warm.on_receive(p)
            warm.close()
            arrivals = [p for p in pk if p.id not in lost] + reps[: len(lost)]
            t0 = time.perf_counter()
            for p in arrivals[:-1]:
                rcv.on_receive(p)
            t1 = time.perf_counter()
            # the k-th row decodes: time the library call itself (the mirror's
            # Python packet objects for k recovered packets are not the product)
            import ctypes
            p = arrivals[-1]
            cap, stride = k + 1024, 2048
            data = (ctypes.c_uint8 * (cap * stride))()
            desc = (L.PacketDesc * cap)()
            nn = ctypes.c_uint32()
            pay = p.payload()
            buf = (ctypes.c_uint8 * len(pay)).from_buffer_copy(pay)
            co = (ctypes.c_uint8 * p.coeff_len).from_buffer_copy(bytes(p.coefficients[: p.coeff_len]))
            t1 = time.perf_counter()
            st_ = rcv._lib.qf_adaptive_on_receive(rcv.handle, p.id, 0, buf, len(pay), co, p.coeff_len, data, stride,
                                                  desc, cap, ctypes.byref(nn))
            t2 = time.perf_counter()
            assert st_ == 0 and nn.value == k
            mv = memoryview(data)
            assert all(bytes(mv[i * stride: i * stride + desc[i].len]) == pk[desc[i].id].payload() for i in range(k))
            entry["receive_us_per_packet"] = round((t1 - t0) / max(1, len(arrivals) - 1) * 1e6, 1)  # (incl. buffers)
            entry["decode_us_kth_packet"] = round((t2 - t1) * 1e6, 1)
            entry["erased"] = len(lost)
            snd.close()
            rcv.close()
        res[mode.name] = entry
        print(mode.name, entry, flush=True)
        fec.close()
    Path(a.out).parent.mkdir(exist_ok=True)
    Path(a.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
