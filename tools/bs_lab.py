#!/usr/bin/env python3
"""Bit-sliced kernel lab: variants of the generated kernels, timed on the GPU.

    python tools/bs_lab.py build            # here: generate + assemble -> tools/lab_build/
    python tools/bs_lab.py run [--G 65536]  # GPU box: load each code object, time it

Variants strip parts of the body (loads, stores, coefficient XORs, all
compute) or change prefetch depth / grid size, to separate the memory and
VALU costs of the real kernel.  Diagnostic only; the library embeds the
unmodified kernels.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
OUT = REPO / "tools" / "lab_build"

VALU = {"v_xor", "v_andk", "v_lshl", "v_lshr", "v_mov", "v_movk", "v_xor3", "v_bitsel_s"}
# address arithmetic (kept by "nodata" even where the register is reused:
# the LU record pointer lives in the accumulator range after the row loop)
ADDR_OPS = {"v_movs", "v_mad64_s", "v_mad64_k", "v_add64_s", "v_cndmask", "v_bfe", "v_readfirstlane"}


def variant_ops(bs, spec, flags):
    ops = bs.generate(spec)
    body = next(n for n, op in enumerate(ops) if op.name == "label" and op.args[0] == ".Lbody")
    acc_lo, acc_hi = spec.acc0, spec.acc0 + 8 * spec.nacc
    ring_lo, ring_hi = spec.ring0, spec.ring0 + 8 * spec.nbuf
    out = []
    for n, op in enumerate(ops):
        # notables: the prologue's split-table copy into LDS dropped (timing
        # only: an upper bound on what loading the tables later could save)
        if "notables" in flags and n < body and (op.name == "ds_write_b128" or
                                                 (op.name == "load16" and 48 <= op.args[0] < 80)):
            continue
        if n > body:
            if "noload" in flags and op.name in ("load16", "load16_lds", "s_waitcnt_vm"):
                continue
            # norowload: only the payload row loads (into the row ring) dropped;
            # slot maps, LU records and rank quads still load
            if "norowload" in flags and op.name in ("load16", "load16_lds") and ring_lo <= op.args[0] < ring_hi:
                continue
            if "nostore" in flags and op.name in ("store16", "store_byte"):
                continue
            if "nocoeff" in flags and op.name in ("v_xor", "v_xor3", "v_mov", "v_movk") and acc_lo <= op.args[0] < acc_hi:
                continue
            if "nocompute" in flags and op.name in VALU:
                continue
            # nodata: every VALU op writing a row-ring or accumulator register
            # dropped (the row loop's transposes, butterflies, folds): the
            # loads and their addressing stay -- the access pattern alone
            if ("nodata" in flags and op.name.startswith("v_") and op.name not in ADDR_OPS and op.args
                    and isinstance(op.args[0], int)
                    and (acc_lo <= op.args[0] < acc_hi or ring_lo <= op.args[0] < ring_hi)):
                continue
        out.append(op)
    # sync:N / synclu: s_barrier after every N-th row wait of the body and
    # (both) after every drained LDS wait (the LU columns' ends), so the
    # workgroup's waves run the same code at about the same time and share
    # its instruction fetches (timing only: the decode's waves exchange no
    # data, so a barrier pairs any two positions safely)
    syncn = next((int(f.split(":")[1]) for f in flags if f.startswith("sync:")), 0)
    if syncn or "synclu" in flags:
        body_at = next(n for n, op in enumerate(out) if op.name == "label" and op.args[0] == ".Lbody")
        synced, nvm = [], 0
        for n, op in enumerate(out):
            synced.append(op)
            if n <= body_at:
                continue
            if op.name == "s_waitcnt_vm" and syncn:
                nvm += 1
                if nvm % syncn == 0:
                    synced.append(bs.Op("s_barrier", ()))
            elif op.name == "s_waitcnt_lgkm_n" and op.args == (0,):
                synced.append(bs.Op("s_barrier", ()))
        out = synced
    for f in flags:   # sched:N -- bs_sched list scheduling, N slots producer -> consumer
        if f.startswith("sched:"):
            from quicfuscate_amd import bs_sched
            out = bs_sched.schedule(out, int(f.split(":")[1]))
    return out


ALL = 1 << 20  # blocks per CU beyond residency: one item per wave
VARIANTS = [
    # round 5ai: prefetch depth of the FFT encode (pd 3 = 240 VGPRs, 2 = 232,
    # 1 = 224: at <= 224 two encode waves leave a 64-VGPR wave slot on the SIMD
    # for the decode's acceptance pass running beside it)
    ("v_warm", 64, 16, 3, ("st:nt", "ztail", "fft:8"), ALL),
    ("v_pd3", 64, 16, 3, ("st:nt", "ztail", "fft:8"), ALL),
    ("v_pd2", 64, 16, 2, ("st:nt", "ztail", "fft:8"), ALL),
    ("v_pd1", 64, 16, 1, ("st:nt", "ztail", "fft:8"), ALL),
    ("v_pd3_2", 64, 16, 3, ("st:nt", "ztail", "fft:8"), ALL),
    ("v_pd2_2", 64, 16, 2, ("st:nt", "ztail", "fft:8"), ALL),
    ("v_pd1_2", 64, 16, 1, ("st:nt", "ztail", "fft:8"), ALL),
]
VARIANTS_R05G = [
    # round 5g: VALU list scheduling (bs_sched, "sched:N") of the FFT encode
    ("u_warm", 64, 16, 3, ("st:nt", "ztail", "fft:8"), ALL),
    ("u_lib", 64, 16, 3, ("st:nt", "ztail", "fft:8"), ALL),
    ("u_s2", 64, 16, 3, ("st:nt", "ztail", "fft:8", "sched:2"), ALL),
    ("u_s3", 64, 16, 3, ("st:nt", "ztail", "fft:8", "sched:3"), ALL),
    ("u_s4", 64, 16, 3, ("st:nt", "ztail", "fft:8", "sched:4"), ALL),
    ("u_lib_2", 64, 16, 3, ("st:nt", "ztail", "fft:8"), ALL),
    ("u_s3_2", 64, 16, 3, ("st:nt", "ztail", "fft:8", "sched:3"), ALL),
]
VARIANTS_R04D = [
    # round 4d: 64-bit-shift transposes in the (HBM-bound) FFT encode
    ("t_warm", 64, 16, 3, ("st:nt", "ztail", "fft:8"), ALL),
    ("t_lib", 64, 16, 3, ("st:nt", "ztail", "fft:8"), ALL),
    ("t_s64", 64, 16, 3, ("st:nt", "ztail", "fft:8", "s64"), ALL),
    ("t_s64_noload", 64, 16, 3, ("noload", "st:nt", "ztail", "fft:8", "s64"), ALL),
    ("t_noload", 64, 16, 3, ("noload", "st:nt", "ztail", "fft:8"), ALL),
    ("t_lib_2", 64, 16, 3, ("st:nt", "ztail", "fft:8"), ALL),
    ("t_s64_2", 64, 16, 3, ("st:nt", "ztail", "fft:8", "s64"), ALL),
]
VARIANTS_R04B = [
    # round 4b: source rows as pool blocks of round_up(L, 128) bytes ("srs:1280":
    # every row starts on a 128-B line; the reference keeps each packet in its
    # own 4,096-B pool block, optimize.rs:139, 440-530) against dense 1,200-B rows
    ("s_warm", 64, 16, 3, ("st:nt", "ztail", "fft:8"), ALL),
    ("s_dense", 64, 16, 3, ("st:nt", "ztail", "fft:8"), ALL),
    ("s_1280", 64, 16, 3, ("st:nt", "ztail", "fft:8", "srs:1280"), ALL),
    ("s_dense_reads", 64, 16, 3, ("nostore", "st:nt", "ztail", "fft:8"), ALL),
    ("s_1280_reads", 64, 16, 3, ("nostore", "st:nt", "ztail", "fft:8", "srs:1280"), ALL),
    ("s_1280_nt", 64, 16, 3, ("ld:nt", "st:nt", "ztail", "fft:8", "srs:1280"), ALL),
    ("s_1280_pd4", 64, 16, 4, ("st:nt", "ztail", "fft:8", "srs:1280"), ALL),
    ("s_dense_2", 64, 16, 3, ("st:nt", "ztail", "fft:8"), ALL),
    ("s_1280_2", 64, 16, 3, ("st:nt", "ztail", "fft:8", "srs:1280"), ALL),
]
VARIANTS_R04A = [
    # round 4: where the encode's 8 % read over-fetch comes from (VERDICT r03
    # item 2).  Run under rocprofv3 --pmc FETCH_SIZE: every variant has its own
    # kernel symbol.  Non-temporal loads drop a row's boundary line before the
    # next row (or the neighbouring item) reads it; the default policy keeps
    # it in L2.  L:1024 rows are line-aligned (no shared lines at all): the
    # FETCH_SIZE calibration of this access pattern.
    ("e_warm", 64, 16, 3, ("ld:nt", "st:nt", "ztail", "fft:8"), ALL),
    ("e_nt", 64, 16, 3, ("ld:nt", "st:nt", "ztail", "fft:8"), ALL),
    ("e_lddef", 64, 16, 3, ("st:nt", "ztail", "fft:8"), ALL),
    ("e_nt_reads", 64, 16, 3, ("nostore", "ld:nt", "st:nt", "ztail", "fft:8"), ALL),
    ("e_lddef_reads", 64, 16, 3, ("nostore", "st:nt", "ztail", "fft:8"), ALL),
    ("e_nt_1024_reads", 64, 16, 3, ("nostore", "ld:nt", "st:nt", "ztail", "fft:8", "L:1024"), ALL),
    ("e_lddef_1024_reads", 64, 16, 3, ("nostore", "st:nt", "ztail", "fft:8", "L:1024"), ALL),
    ("e_nt_2", 64, 16, 3, ("ld:nt", "st:nt", "ztail", "fft:8"), ALL),
    ("e_lddef_2", 64, 16, 3, ("st:nt", "ztail", "fft:8"), ALL),
]
VARIANTS_R03Z = [
    # round 3z: dense 1,200-B repair rows with the line-aligned item layout
    # (no zero-tail bytes: 1.3 % less traffic) against the zero-tail default
    ("z_warm", 64, 16, 3, ("ld:nt", "st:nt", "ztail", "fft:8"), ALL),
    ("z_ztail", 64, 16, 3, ("ld:nt", "st:nt", "ztail", "fft:8"), ALL),
    ("z_dense", 64, 16, 3, ("ld:nt", "st:nt", "pad80", "fft:8"), ALL),
    ("z_dense_stdef", 64, 16, 3, ("ld:nt", "pad80", "fft:8"), ALL),
    ("z_ztail_2", 64, 16, 3, ("ld:nt", "st:nt", "ztail", "fft:8"), ALL),
    ("z_dense_2", 64, 16, 3, ("ld:nt", "st:nt", "pad80", "fft:8"), ALL),
]
VARIANTS_R03B = [
    # round 3b: rows staged in LDS ("lds:<slots per wave>", global_load_lds_dwordx4)
    ("warm", 64, 16, 3, ("ld:nt", "st:nt", "ztail", "fft:8"), ALL),
    ("fft_pd3", 64, 16, 3, ("ld:nt", "st:nt", "ztail", "fft:8"), ALL),
    ("fft_l6", 64, 16, 3, ("ld:nt", "st:nt", "ztail", "fft:8", "lds:6"), ALL),
    ("fft_l8", 64, 16, 3, ("ld:nt", "st:nt", "ztail", "fft:8", "lds:8"), ALL),
    ("fft_l9", 64, 16, 3, ("ld:nt", "st:nt", "ztail", "fft:8", "lds:9"), ALL),
    ("fft_l9_nocompute", 64, 16, 3, ("nocompute", "ld:nt", "st:nt", "ztail", "fft:8", "lds:9"), ALL),
    ("fft_l9_nostore", 64, 16, 3, ("nostore", "ld:nt", "st:nt", "ztail", "fft:8", "lds:9"), ALL),
    ("fft_l9_stdef", 64, 16, 3, ("ld:nt", "ztail", "fft:8", "lds:9"), ALL),
    ("fft_l9_lddef", 64, 16, 3, ("st:nt", "ztail", "fft:8", "lds:9"), ALL),
    ("fft_pd3_2", 64, 16, 3, ("ld:nt", "st:nt", "ztail", "fft:8"), ALL),
    ("fft_l9_2", 64, 16, 3, ("ld:nt", "st:nt", "ztail", "fft:8", "lds:9"), ALL),
]
VARIANTS_R03A = [
    # round 3: the additive-FFT encode ("fft:<ch>", "defer:<rows>")
    ("warm", 64, 16, 3, ("ld:nt", "st:nt", "ztail"), ALL),
    ("classic", 64, 16, 3, ("ld:nt", "st:nt", "ztail"), ALL),
    ("fft_pd3", 64, 16, 3, ("ld:nt", "st:nt", "ztail", "fft:8"), ALL),
    ("fft_pd4", 64, 16, 4, ("ld:nt", "st:nt", "ztail", "fft:8"), ALL),
    ("fft_pd5", 64, 16, 5, ("ld:nt", "st:nt", "ztail", "fft:8"), ALL),
    ("fft_pd3_d2", 64, 16, 3, ("ld:nt", "st:nt", "ztail", "fft:8", "defer:2"), ALL),
    ("fft_pd4_d1", 64, 16, 4, ("ld:nt", "st:nt", "ztail", "fft:8", "defer:1"), ALL),
    ("fft_pd2_d3", 64, 16, 2, ("ld:nt", "st:nt", "ztail", "fft:8", "defer:3"), ALL),
    ("fft_nocompute", 64, 16, 3, ("nocompute", "ld:nt", "st:nt", "ztail", "fft:8"), ALL),
    ("fft_noload", 64, 16, 3, ("noload", "ld:nt", "st:nt", "ztail", "fft:8"), ALL),
    ("fft_nostore", 64, 16, 3, ("nostore", "ld:nt", "st:nt", "ztail", "fft:8"), ALL),
    ("classic_2", 64, 16, 3, ("ld:nt", "st:nt", "ztail"), ALL),
    ("fft_pd3_2", 64, 16, 3, ("ld:nt", "st:nt", "ztail", "fft:8"), ALL),
]
VARIANTS_R02 = [
    # name, k, r, pd, flags, blocks_per_cu  (flags: "plain" = no v_bitop3 xor;
    # "nobfi" = classic 6-op delta swaps; "noremap" = no XCD-aware item order;
    # "ld:/st:<bits>" cache policy; "L:<n>" payload bytes; "dst:wide" 2048-B
    # repair rows; "ztail" padded lane space + zero tail, 128-B repair rows;
    # "nocompute" drops every VALU op of the body (incl. v_bitop3))
    ("warm", 64, 16, 3, ("ld:nt", "st:nt"), ALL),
    ("full", 64, 16, 3, ("ld:nt", "st:nt"), ALL),
    ("full_ztail", 64, 16, 3, ("ld:nt", "st:nt", "ztail"), ALL),
    ("mem_ztail", 64, 16, 3, ("nocompute", "ld:nt", "st:nt", "ztail"), ALL),
    ("writeonly_ztail", 64, 16, 3, ("nocompute", "noload", "ld:nt", "st:nt", "ztail"), ALL),
    ("full_ztail_pd2", 64, 16, 2, ("ld:nt", "st:nt", "ztail"), ALL),
    ("full_ztail_pd4", 64, 16, 4, ("ld:nt", "st:nt", "ztail"), ALL),
    ("full_ztail_stdef", 64, 16, 3, ("ld:nt", "ztail"), ALL),
    ("full_ztail_noremap", 64, 16, 3, ("ld:nt", "st:nt", "ztail", "noremap"), ALL),
    ("full_2", 64, 16, 3, ("ld:nt", "st:nt"), ALL),
    ("full_ztail_2", 64, 16, 3, ("ld:nt", "st:nt", "ztail"), ALL),
]


def build():
    from quicfuscate_amd import bs_codegen as bs
    from quicfuscate_amd.build_lib import assemble

    OUT.mkdir(parents=True, exist_ok=True)
    for old in OUT.glob("lab_*"):
        old.unlink()
    manifest = []
    for name, k, r, pd, flags, bpc in VARIANTS:
        ld = next((f[3:] for f in flags if f.startswith("ld:")), "")
        st = next((f[3:] for f in flags if f.startswith("st:")), "")
        spec = bs.KernelSpec(k, r, pd, xor3="plain" not in flags, ld_policy=ld, st_policy=st,
                             bfi_transpose="s64" if "s64" in flags else "nobfi" not in flags,
                             xcd_remap="noremap" not in flags,
                             fft=next((int(f[4:]) for f in flags if f.startswith("fft:")), 0),
                             fft_defer=next((int(f[6:]) for f in flags if f.startswith("defer:")), 0),
                             lds_rows=next((int(f[4:]) for f in flags if f.startswith("lds:")), 0))
        text = bs.emit_asm(spec, variant_ops(bs, spec, set(flags)))
        h = assemble(f"lab_{name}", text.replace(spec.name, f"lab_{name}"), OUT)
        Lv = next((int(f[2:]) for f in flags if f.startswith("L:")), 1200)
        manifest.append({"name": name, "k": k, "r": r, "pd": pd, "flags": list(flags), "blocks_per_cu": bpc, "L": Lv,
                         "hsaco": h.name, "symbol": f"lab_{name}", "vgprs": spec.next_free_vgpr})
        print(name, h.stat().st_size)
    (OUT / "manifest.json").write_text(json.dumps(manifest, indent=1))


def run(G: int, reps: int):
    import torch

    from quicfuscate_amd import bs_codegen as bs

    hip = ctypes.CDLL(str(Path(torch.__file__).parent / "lib" / "libamdhip64.so"))
    dev = torch.device("cuda")
    manifest = json.loads((OUT / "manifest.json").read_text())
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    kmax, rmax, Lmax = 64, 16, 1280
    src = torch.randint(0, 256, (G * kmax * Lmax,), dtype=torch.uint8, device=dev)
    dst = torch.empty(G * 32768, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream()
    res = {}
    for m in manifest:
        k, r, L = m["k"], m["r"], m["L"]
        mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
        data = (OUT / m["hsaco"]).read_bytes()
        buf = ctypes.create_string_buffer(data, len(data))
        assert hip.hipModuleLoadData(ctypes.byref(mod), buf) == 0
        assert hip.hipModuleGetFunction(ctypes.byref(fn), mod, m["symbol"].encode()) == 0
        zt = "ztail" in m["flags"]
        # pad80: the padded lane space (items line-aligned) but dense repair rows
        # of L bytes and no zero tail (the padding lanes store nothing)
        Lv = bs.padded_units(L) if (zt or "pad80" in m["flags"]) else None
        _, _, n_items = bs.launch_geometry(L, G, Lv)
        blocks = min((n_items + 3) // 4, ncu * m["blocks_per_cu"])
        wide = "dst:wide" in m["flags"]
        drs, dgs = (2048, 32768) if wide else ((16 * Lv, 16 * Lv * r) if zt else (L, r * L))
        srs = next((int(f[4:]) for f in m["flags"] if f.startswith("srs:")), L)
        ka = bs.kernargs(src.data_ptr(), dst.data_ptr(), k * srs, dgs, srs, drs, L, G, blocks * 4, Lv=Lv, zero_tail=zt)
        kbuf = ctypes.create_string_buffer(ka, len(ka))
        size = ctypes.c_size_t(len(ka))
        extra = (ctypes.c_void_p * 5)(1, ctypes.cast(kbuf, ctypes.c_void_p), 2,
                                     ctypes.cast(ctypes.pointer(size), ctypes.c_void_p), 3)

        def launch():
            e = hip.hipModuleLaunchKernel(fn, blocks, 1, 1, 256, 1, 1, 0, ctypes.c_void_p(stream.cuda_stream),
                                          None, extra)
            assert e == 0, e

        launch()
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record(stream)
        for _ in range(reps):
            launch()
        t1.record(stream)
        torch.cuda.synchronize()
        ms = t0.elapsed_time(t1) / reps
        gb = G * (k + r) * L / (ms / 1e3) / 1e9
        res[m["name"]] = {"ms": round(ms, 4), "GBps_alg": round(gb, 1), "pd": m["pd"], "flags": m["flags"],
                          "blocks_per_cu": m["blocks_per_cu"], "vgprs": m["vgprs"]}
        print(m["name"], res[m["name"]], flush=True)
        hip.hipModuleUnload(mod)
    return res


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["build", "run"])
    ap.add_argument("--G", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", default="gpurun_out/bs_lab.json")
    a = ap.parse_args()
    if a.cmd == "build":
        build()
    else:
        r = run(a.G, a.reps)
        Path(a.out).parent.mkdir(exist_ok=True)
        Path(a.out).write_text(json.dumps(r, indent=1))
