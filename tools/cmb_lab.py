#!/usr/bin/env python3
"""Payload-pass lab (gfx950): variants of the bit-sliced payload kernel with
wave-uniform runtime coefficients (bs_codegen "cmb") timed on
synthetic C5-sized batches -- e syndrome rows in, e recovered rows out per
generation, 9,000-B rows, random coefficient records -- with HIP events.

    python tools/cmb_lab.py build     # here: tools/lab_build/cmb_*.hsaco
    python tools/cmb_lab.py run       # GPU box (tools/gpurun_lab.sh)

Each variant's output is compared with the first variant of the same (e,
passes) case (the library's kernel), so timing-only lab flags show as
matches_base False."""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
OUT = REPO / "tools" / "lab_build"
L = 9000
RS = 9008

# (name, e, R, pass_major, KernelSpec keyword overrides); the first variant of
# each e is the reference the others' outputs are compared with
VARIANTS = [
    # round 6d: with the jump products, does the syndrome re-read bound the
    # pass-major pass? pass-major against the XCD interleave, both jump
    ("e39_pm_j3", 39, 16, True, {"cmb_lean": True, "cmb_jump": 3}),
    ("e39_xcd_j3", 39, 16, True, {"cmb_lean": True, "cmb_jump": 3, "pm_xcd": True}),
    ("e48_pm_j3", 48, 16, True, {"cmb_lean": True, "cmb_jump": 3}),
    ("e48_xcd_j3", 48, 16, True, {"cmb_lean": True, "cmb_jump": 3, "pm_xcd": True}),
    ("e59_pm_j3", 59, 16, True, {"cmb_lean": True, "cmb_jump": 3}),
    ("e59_xcd_j3", 59, 16, True, {"cmb_lean": True, "cmb_jump": 3, "pm_xcd": True}),
    ("e32_pm_j3", 32, 16, True, {"cmb_lean": True, "cmb_jump": 3}),
    ("e32_xcd_j3", 32, 16, True, {"cmb_lean": True, "cmb_jump": 3, "pm_xcd": True}),
    ("e39_pm_j3_2", 39, 16, True, {"cmb_lean": True, "cmb_jump": 3}),
    ("e39_xcd_j3_2", 39, 16, True, {"cmb_lean": True, "cmb_jump": 3, "pm_xcd": True}),
    ("e48_pm_j3_2", 48, 16, True, {"cmb_lean": True, "cmb_jump": 3}),
    ("e48_xcd_j3_2", 48, 16, True, {"cmb_lean": True, "cmb_jump": 3, "pm_xcd": True}),
]


LAB_KEYS = ("bpc", "split", "rows")


def make_spec(bs, R, pm, kw):
    return bs.KernelSpec(0, R, 3, "cmb", pass_major=pm, **{a: b for a, b in kw.items() if a not in LAB_KEYS})


def build():
    from quicfuscate_amd import bs_codegen as bs
    from quicfuscate_amd.build_lib import assemble

    OUT.mkdir(parents=True, exist_ok=True)
    for old in OUT.glob("cmb_*"):
        old.unlink()
    manifest = []
    for name, e, R, pm, kw in VARIANTS:
        spec = make_spec(bs, R, pm, kw)
        text = bs.emit_asm(spec, bs.generate(spec))
        h = assemble(f"cmb_{name}", text.replace(spec.name, f"cmb_{name}"), OUT)
        manifest.append({"name": name, "e": e, "R": R, "pm": pm, "kw": {k: (list(v) if isinstance(v, tuple) else v) for k, v in kw.items()},
                         "hsaco": h.name, "symbol": f"cmb_{name}", "vgprs": spec.next_free_vgpr})
        print(name, spec.next_free_vgpr, h.stat().st_size, flush=True)
    (OUT / "cmb_manifest.json").write_text(json.dumps(manifest, indent=1))


def run(nbytes: float, reps: int):
    import numpy as np
    import torch

    from quicfuscate_amd import bs_codegen as bs

    hip = ctypes.CDLL(str(Path(torch.__file__).parent / "lib" / "libamdhip64.so"))
    manifest = json.loads((OUT / "cmb_manifest.json").read_text())
    stream = torch.cuda.current_stream()
    idxtab = torch.from_numpy(bs.cmb_index_table().reshape(-1).view(np.uint8).copy()).cuda()
    res, cur, base_out = {}, None, {}
    for m in manifest:
        e = m["e"]
        nr = m["kw"].get("rows", e)   # input rows per generation (default: e syndromes)
        G = max(1, int(nbytes // (nr * L)))
        P = (e + 15) // 16
        cgs = (nr + 1) * 16
        PS = G * cgs
        if cur != (e, nr):
            g = torch.Generator(device="cuda").manual_seed(e)
            rows = torch.randint(0, 256, (G * nr * RS,), dtype=torch.uint8, device="cuda", generator=g)
            rec = torch.randint(0, 256, (P * PS,), dtype=torch.uint8, device="cuda", generator=g)
            n_out = torch.full((G,), e, dtype=torch.int32, device="cuda")
            bound = torch.full((G,), nr, dtype=torch.int32, device="cuda")
            dst = torch.empty(G * e * RS, dtype=torch.uint8, device="cuda")
            cur = (e, nr)
        mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
        data = (OUT / m["hsaco"]).read_bytes()
        buf = ctypes.create_string_buffer(data, len(data))
        assert hip.hipModuleLoadData(ctypes.byref(mod), buf) == 0
        assert hip.hipModuleGetFunction(ctypes.byref(fn), mod, m["symbol"].encode()) == 0
        Lu = (L + 15) // 16
        ipg = ((Lu + 1) // 2 + 63) // 64
        blocks = min((G * ipg + 3) // 4, m["kw"].get("bpc", 2) * 256)
        passes = P if m["pm"] else 1
        xcd = bool(m["kw"].get("pm_xcd"))
        if xcd:   # slots in groups of 8 (one per XCD)
            blocks = (blocks + 7) // 8 * 8
        split = m["kw"].get("split", 1)
        R = m["R"]
        n_outs = [n_out] if split == 1 else [torch.full((G,), max(0, e - R * i), dtype=torch.int32, device="cuda")
                                             for i in range(split)]
        extras, keep = [], []
        for i in range(split):   # launch i: record bytes R i.., output rows R i..
            ka, _ = bs.cmb_kernargs(rows.data_ptr(), dst.data_ptr() + R * i * RS, nr * RS, e * RS, RS, RS,
                                    rec.data_ptr() + R * i, cgs, 0, n_outs[i].data_ptr(), bound.data_ptr(),
                                    idxtab.data_ptr(), L, G, 4 * blocks, pass_stride=PS,
                                    pm_xcd_passes=passes if xcd else 0)
            kbuf = ctypes.create_string_buffer(ka, len(ka))
            size = ctypes.c_size_t(len(ka))
            keep += [kbuf, size]
            extras.append((ctypes.c_void_p * 5)(1, ctypes.cast(kbuf, ctypes.c_void_p), 2,
                                                ctypes.cast(ctypes.pointer(size), ctypes.c_void_p), 3))

        def launch():
            for extra in extras:
                err = hip.hipModuleLaunchKernel(fn, blocks * passes, 1, 1, 256, 1, 1, 0,
                                                ctypes.c_void_p(stream.cuda_stream), None, extra)
                assert err == 0, err

        dst.fill_(0xA5)
        launch()
        torch.cuda.synchronize()
        if (e, nr) not in base_out:
            base_out[(e, nr)] = dst.clone()
        ok = bool(torch.equal(dst, base_out[(e, nr)]))
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record(stream)
        for _ in range(reps):
            launch()
        t1.record(stream)
        torch.cuda.synchronize()
        ms = t0.elapsed_time(t1) / reps
        res[m["name"]] = {"ms": round(ms, 4), "G": G, "e": e, "passes": passes, "matches_base": ok,
                          "vgprs": m["vgprs"], "kw": m["kw"],
                          "indexed_xor_per_simd_per_ns": round(G * ipg * nr * e * 16 / (ms * 1e6) / 1024, 3)}
        print(m["name"], res[m["name"]], flush=True)
        hip.hipModuleUnload(mod)
    return res


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["build", "run"])
    ap.add_argument("--bytes", type=float, default=2e9, help="syndrome bytes per case (G = bytes / (e L))")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", default="gpurun_out/cmb_lab.json")
    a = ap.parse_args()
    if a.cmd == "build":
        build()
    else:
        r = run(a.bytes, a.reps)
        Path(a.out).parent.mkdir(parents=True, exist_ok=True)
        Path(a.out).write_text(json.dumps(r, indent=1))
