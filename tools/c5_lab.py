#!/usr/bin/env python3
"""C5 pass-kernel lab: variants of the merged multi-pass encode (MergedSpec)
at the C5 jumbo shapes, timed on the GPU and checked against the library's
encode of the same batch.

    python tools/c5_lab.py build                      # here: generate + assemble -> tools/lab_build/c5_*
    python tools/c5_lab.py run [--bytes 1e9]          # GPU box

Variant kinds: "N" additive-FFT coset passes (lch_fft.coset_passes), "M"
plain passes split into `npass` balanced ranges.  Diagnostic only.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
OUT = REPO / "tools" / "lab_build"
L_JUMBO, RS, DRS = 9000, 9008, 9088

# (name, k, rt, kind, npass (M), KernelSpec keyword overrides)
VARIANTS = [
    # round 5bi: single-pass C5 codes -- the library's plain pass ("S") against
    # the hybrid additive-FFT pass (fft=8: sources past 2^a folded in directly)
    ("s96_warm", 96, 15, "S", 0, {}),
    ("s96_plain", 96, 15, "S", 0, {}),
    ("s96_fft", 96, 15, "S", 0, {"fft": 8, "ld_policy": ""}),
    ("s48_plain", 48, 8, "S", 0, {}),
    ("s48_fft", 48, 8, "S", 0, {"fft": 8, "ld_policy": ""}),
    ("s32_plain", 32, 5, "S", 0, {}),
    ("s32_fft", 32, 5, "S", 0, {"fft": 8, "ld_policy": ""}),
    ("s96_plain_2", 96, 15, "S", 0, {}),
    ("s96_fft_2", 96, 15, "S", 0, {"fft": 8, "ld_policy": ""}),
    ("s48_plain_2", 48, 8, "S", 0, {}),
    ("s48_fft_2", 48, 8, "S", 0, {"fft": 8, "ld_policy": ""}),
]
VARIANTS_R05BF = [
    # round 5bf: (128, 20) -- the library's single plain pass against the
    # additive-FFT coset passes sharing their row work (xchg, with helpers)
    # (the plain pass is not a merged kernel: its time is the bench's block
    # encode, 0.238-0.242 ms at this size, profiles/r05bc_bench_detail.json)
    ("q128_warm", 128, 20, "N", 0, {"xchg": True}),
    ("q128_x", 128, 20, "N", 0, {"xchg": True}),
    ("q128_xh2", 128, 20, "N", 0, {"xchg": True, "helpers": 2, "xchg_early": 3}),
    ("q128_xh2e0", 128, 20, "N", 0, {"xchg": True, "helpers": 2}),
    ("q128_x_2", 128, 20, "N", 0, {"xchg": True}),
    ("q128_xh2_2", 128, 20, "N", 0, {"xchg": True, "helpers": 2, "xchg_early": 3}),
]
VARIANTS_R05AU = [
    # round 5au: each wave issues the loads of its next group's first rows
    # before transforming the current group (KernelSpec.xchg_early rotating slots)
    ("e196_warm", 196, 59, "N", 0, {"xchg": True}),
    ("e196_x", 196, 59, "N", 0, {"xchg": True}),
    ("e196_e3", 196, 59, "N", 0, {"xchg": True, "xchg_early": 3}),
    ("e196_e5", 196, 59, "N", 0, {"xchg": True, "xchg_early": 5}),
    ("e160_x", 160, 48, "N", 0, {"xchg": True}),
    ("e160_e5", 160, 48, "N", 0, {"xchg": True, "xchg_early": 5}),
    ("e196_x_2", 196, 59, "N", 0, {"xchg": True}),
    ("e196_e3_2", 196, 59, "N", 0, {"xchg": True, "xchg_early": 3}),
    ("e196_e5_2", 196, 59, "N", 0, {"xchg": True, "xchg_early": 5}),
    ("e160_x_2", 160, 48, "N", 0, {"xchg": True}),
    ("e160_e5_2", 160, 48, "N", 0, {"xchg": True, "xchg_early": 5}),
]
VARIANTS_R05AT = [
    # round 5at: what the shared-row (196, 59) encode waits on: no row loads
    # (compute, LDS exchange and barriers only) / no VALU data work (loads,
    # LDS exchange, barriers, stores)
    ("z196_warm", 196, 59, "N", 0, {"xchg": True}),
    ("z196_x", 196, 59, "N", 0, {"xchg": True}),
    ("z196_noload", 196, 59, "N", 0, {"xchg": True, "flags": ("noload",)}),
    ("z196_novalu", 196, 59, "N", 0, {"xchg": True, "flags": ("novalu",)}),
    ("z196_x_2", 196, 59, "N", 0, {"xchg": True}),
    ("z196_noload_2", 196, 59, "N", 0, {"xchg": True, "flags": ("noload",)}),
    ("z196_novalu_2", 196, 59, "N", 0, {"xchg": True, "flags": ("novalu",)}),
]
VARIANTS_R05AE = [
    # round 5ae: a producer-only 4th wave in the 3-pass codes' workgroups
    # (merged_spec(xchg=True, helpers=1)): two workgroups then fill a CU's 8
    # wave slots
    ("h160_warm", 160, 48, "N", 0, {"xchg": True}),
    ("h160_x", 160, 48, "N", 0, {"xchg": True}),
    ("h160_xh", 160, 48, "N", 0, {"xchg": True, "helpers": 1}),
    ("h128_x", 128, 39, "N", 0, {"xchg": True}),
    ("h128_xh", 128, 39, "N", 0, {"xchg": True, "helpers": 1}),
    ("h160_x_2", 160, 48, "N", 0, {"xchg": True}),
    ("h160_xh_2", 160, 48, "N", 0, {"xchg": True, "helpers": 1}),
    ("h128_x_2", 128, 39, "N", 0, {"xchg": True}),
    ("h128_xh_2", 128, 39, "N", 0, {"xchg": True, "helpers": 1}),
]
VARIANTS_R05U = [
    # round 5u: the waves of a merged FFT encode share loads, transposes and
    # chunk butterflies through LDS (merged_spec(xchg=True))
    ("x196_warm", 196, 59, "N", 0, {}),
    ("x196_lib", 196, 59, "N", 0, {}),
    ("x196_xchg", 196, 59, "N", 0, {"xchg": True}),
    ("x160_lib", 160, 48, "N", 0, {}),
    ("x160_xchg", 160, 48, "N", 0, {"xchg": True}),
    ("x128_lib", 128, 39, "N", 0, {}),
    ("x128_xchg", 128, 39, "N", 0, {"xchg": True}),
    ("x196_lib_2", 196, 59, "N", 0, {}),
    ("x196_xchg_2", 196, 59, "N", 0, {"xchg": True}),
]
VARIANTS_R05H = [
    # round 5h: what bounds the (196, 59) merged encode: no row loads (compute
    # and stores only) / no VALU data work (loads, addresses, stores only)
    ("b196_warm", 196, 59, "N", 0, {}),
    ("b196_lib", 196, 59, "N", 0, {}),
    ("b196_noload", 196, 59, "N", 0, {"flags": ("noload",)}),
    ("b196_novalu", 196, 59, "N", 0, {"flags": ("novalu",)}),
    ("b196_same", 196, 59, "N", 0, {"flags": ("same",)}),
    ("b196_lib_2", 196, 59, "N", 0, {}),
    ("b196_noload_2", 196, 59, "N", 0, {"flags": ("noload",)}),
    ("b196_novalu_2", 196, 59, "N", 0, {"flags": ("novalu",)}),
]
VARIANTS_R05G = [
    # round 5g: VALU list scheduling of the merged FFT passes (bs_sched)
    ("s196_warm", 196, 59, "N", 0, {}),
    ("s196_lib", 196, 59, "N", 0, {}),
    ("s196_s2", 196, 59, "N", 0, {"sched": 2}),
    ("s196_s3", 196, 59, "N", 0, {"sched": 3}),
    ("s196_s4", 196, 59, "N", 0, {"sched": 4}),
    ("s160_lib", 160, 48, "N", 0, {}),
    ("s160_s3", 160, 48, "N", 0, {"sched": 3}),
    ("s128_lib", 128, 39, "N", 0, {}),
    ("s128_s3", 128, 39, "N", 0, {"sched": 3}),
    ("s196_lib_2", 196, 59, "N", 0, {}),
    ("s196_s3_2", 196, 59, "N", 0, {"sched": 3}),
]
VARIANTS_R04 = [
    ("n160_lib", 160, 48, "N", 0, {}),
    ("n160_c8pd2", 160, 48, "N", 0, {"fft_coset": 8, "pd": 2}),
    ("n160_c8pd3", 160, 48, "N", 0, {"fft_coset": 8, "pd": 3}),
    ("n160_c8lds6", 160, 48, "N", 0, {"fft_coset": 8, "lds_rows": 6}),
    ("n128_c8pd2", 128, 39, "N", 0, {"fft_coset": 8, "pd": 2}),
    ("n196_c8lds4", 196, 59, "N", 0, {"fft_coset": 8, "lds_rows": 4}),
    ("n160_lds6", 160, 48, "N", 0, {"lds_rows": 6}),
    ("n160_lds8", 160, 48, "N", 0, {"lds_rows": 8}),
    ("n160_lds10", 160, 48, "N", 0, {"lds_rows": 10}),
    ("m160_lib", 160, 48, "M", 4, {}),
    ("m160_pd2", 160, 48, "M", 4, {"pd": 2}),
    ("m160_p3", 160, 48, "M", 3, {}),
    ("n160_noload", 160, 48, "N", 0, {"flags": ("noload",)}),
    ("n160_novalu", 160, 48, "N", 0, {"flags": ("novalu",)}),
    ("n160_same", 160, 48, "N", 0, {"flags": ("same",)}),
    ("n160_same_noload", 160, 48, "N", 0, {"flags": ("same", "noload")}),
    ("n196_lib", 196, 59, "N", 0, {}),
    ("n196_lds8", 196, 59, "N", 0, {"lds_rows": 8}),
    ("m196_lib", 196, 59, "M", 4, {}),
    ("n128_lib", 128, 39, "N", 0, {}),
    ("n128_lds8", 128, 39, "N", 0, {"lds_rows": 8}),
    ("m128_lib", 128, 39, "M", 2, {}),
    ("m128_p3pd2", 128, 39, "M", 3, {"pd": 2}),
]


def make_spec(bs, k, rt, kind, npass, kw):
    from quicfuscate_amd import lch_fft

    pd = kw.get("pd", 3)
    extra = {x: v for x, v in kw.items() if x not in ("pd", "flags", "xchg", "helpers")}
    if kind == "S":   # one plain / hybrid-FFT pass (4 one-item waves per workgroup, as the library)
        return bs.KernelSpec(k, rt, pd, "enc", **extra)
    if kind == "N":
        R = extra.get("fft_coset", 16)
        passes = [bs.KernelSpec(k, rp, pd, "enc", fft=8, ld_policy="", r_total=rt, j0=j0, **extra)
                  for j0, rp in lch_fft.coset_passes(k, rt, R)]
        return bs.merged_spec(passes, xchg=bool(kw.get("xchg")), helpers=kw.get("helpers", 0))
    else:
        cuts = [rt * p // npass for p in range(npass + 1)]
        passes = [bs.KernelSpec(k, cuts[p + 1] - cuts[p], pd, "enc", r_total=rt, j0=cuts[p], **extra)
                  for p in range(npass)]
    return bs.merged_spec(passes)


VALU = {"v_xor", "v_xor3", "v_mov", "v_movk", "v_bitsel_s", "v_bitop3", "v_lshl64", "v_lshr64", "v_bfi", "v_and_s",
        "v_perm"}


def variant_ops(bs, ms, flags):
    """noload: no row loads / load waits in the pass bodies; novalu: no
    XOR / move / select work in them (loads, addresses, stores kept); same:
    every wave runs pass 0 (no dispatch: one body's code for all waves)."""
    ops = bs.generate(ms)
    out, in_body = [], False
    for n, op in enumerate(ops):
        if op.name == "label" and op.args[0].startswith(".LP") and op.args[0].endswith("body"):
            in_body = True
        if op.name == "label" and op.args[0].startswith(".Lpass"):
            in_body = False
        if "same" in flags and op.name in ("s_cmp_lg_k_br", "s_far_jump") and str(op.args[0]).startswith((".Lnpass", ".Lpass")):
            continue
        if in_body and "noload" in flags and op.name in ("load16", "load16_lds", "s_waitcnt_vm"):
            continue
        if in_body and "novalu" in flags and (op.name in VALU or (op.name.startswith("v_") and op.name not in
                                                                   ("v_add64_s", "v_add64_v", "v_mad64_k",
                                                                    "v_mad64_s", "v_movs", "v_readfirstlane",
                                                                    "v_add_s", "v_addk", "v_cmp_eq_s", "v_cmp_gt_s"))):
            continue
        out.append(op)
    return out


def build():
    from quicfuscate_amd import bs_codegen as bs
    from quicfuscate_amd.build_lib import assemble

    OUT.mkdir(parents=True, exist_ok=True)
    for old in OUT.glob("c5_*"):
        old.unlink()
    manifest = []
    for name, k, rt, kind, npass, kw in VARIANTS:
        ms = make_spec(bs, k, rt, kind, npass, kw)
        text = bs.emit_asm(ms, variant_ops(bs, ms, set(kw.get("flags", ()))))
        h = assemble(f"c5_{name}", text.replace(ms.name, f"c5_{name}"), OUT)
        manifest.append({"name": name, "k": k, "rt": rt, "kind": kind, "npass": npass, "kw": kw, "waves": getattr(ms, "waves", 4),
                         "hsaco": h.name, "symbol": f"c5_{name}", "vgprs": ms.next_free_vgpr, "lds": ms.lds_bytes})
        print(name, getattr(ms, "waves", 4), ms.next_free_vgpr, ms.lds_bytes, h.stat().st_size, flush=True)
    (OUT / "c5_manifest.json").write_text(json.dumps(manifest, indent=1))


def run(nbytes: float, reps: int):
    import torch

    from quicfuscate_amd import bs_codegen as bs
    from quicfuscate_amd import fec as qf

    hip = ctypes.CDLL(str(Path(torch.__file__).parent / "lib" / "libamdhip64.so"))
    manifest = json.loads((OUT / "c5_manifest.json").read_text())
    ctx = qf.default_context()
    stream = torch.cuda.current_stream()
    res = {}
    cur = None
    for m in manifest:
        k, rt = m["k"], m["rt"]
        G = max(1, int(nbytes // (k * L_JUMBO)))
        if cur != (k, rt):
            src = torch.randint(0, 256, (G * k * RS,), dtype=torch.uint8, device="cuda")
            ref = torch.empty(G * rt * DRS, dtype=torch.uint8, device="cuda")
            qf.encode_batch(src, ref, k, rt, L_JUMBO, src_row_stride=RS, src_gen_stride=k * RS, rep_row_stride=DRS,
                            rep_gen_stride=rt * DRS, G=G, zero_tail=True, ctx=ctx)
            ctx.sync()
            dst = torch.empty_like(ref)
            cur = (k, rt)
        mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
        data = (OUT / m["hsaco"]).read_bytes()
        buf = ctypes.create_string_buffer(data, len(data))
        assert hip.hipModuleLoadData(ctypes.byref(mod), buf) == 0
        assert hip.hipModuleGetFunction(ctypes.byref(fn), mod, m["symbol"].encode()) == 0
        Lv = bs.padded_units(L_JUMBO)
        _, _, n_items = bs.launch_geometry(L_JUMBO, G, Lv)
        blocks = n_items
        stride = blocks
        if m["kind"] == "S":   # one item per wave, 4-wave workgroups, item stride in waves
            blocks = (n_items + 3) // 4
            stride = 4 * blocks
        ka = bs.kernargs(src.data_ptr(), dst.data_ptr(), k * RS, rt * DRS, RS, DRS, L_JUMBO, G, stride, Lv=Lv,
                         zero_tail=True)
        kbuf = ctypes.create_string_buffer(ka, len(ka))
        size = ctypes.c_size_t(len(ka))
        extra = (ctypes.c_void_p * 5)(1, ctypes.cast(kbuf, ctypes.c_void_p), 2,
                                     ctypes.cast(ctypes.pointer(size), ctypes.c_void_p), 3)

        def launch():
            e = hip.hipModuleLaunchKernel(fn, blocks, 1, 1, 64 * m["waves"], 1, 1, 0,
                                          ctypes.c_void_p(stream.cuda_stream), None, extra)
            assert e == 0, e

        dst.fill_(0xA5)
        launch()
        torch.cuda.synchronize()
        ok = bool(torch.equal(dst, ref))
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record(stream)
        for _ in range(reps):
            launch()
        t1.record(stream)
        torch.cuda.synchronize()
        ms = t0.elapsed_time(t1) / reps
        gib = G * (k + rt) * L_JUMBO / (ms / 1e3) / 2**30
        res[m["name"]] = {"ms": round(ms, 4), "GiBps_alg": round(gib, 1), "G": G, "matches_library": ok,
                          "waves": m["waves"], "vgprs": m["vgprs"], "lds": m["lds"], "kw": m["kw"]}
        print(m["name"], res[m["name"]], flush=True)
        hip.hipModuleUnload(mod)
    return res


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["build", "run"])
    ap.add_argument("--bytes", type=float, default=1e9)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default="gpurun_out/c5_lab.json")
    a = ap.parse_args()
    if a.cmd == "build":
        build()
    else:
        r = run(a.bytes, a.reps)
        Path(a.out).parent.mkdir(exist_ok=True)
        Path(a.out).write_text(json.dumps(r, indent=1))
