#!/usr/bin/env python3
"""BASELINE C5 throughput on the MI355X (diagnostic beside bench.py): the
adaptive sliding-window shapes of SURVEY 8(d) -- k 32..196, r = ceil(k*ratio)-k,
9000-byte jumbo payloads -- in block mode (independent generations) and
sliding mode (one window per source packet: generation stride = row stride),
encode and decode at 20 % source loss, device-resident, HIP-event kernel
times.  Algorithmic bytes: block encode (k + r) L per generation,
decode (k + e) L, sliding encode (1 + r) L per window -- compute-bound by
construction, so its VALU issue fraction is reported beside the HBM one.

    python tools/bench_c5.py [--bytes 1e9] [--mixed-bytes 4e9] [--out gpurun_out/c5_bench.json] [--mixed-only]

bench.py runs the same legs (c5_bench) as the `c5` object of its line.

The first leg is one heterogeneous batch of all shapes (qf_encode_batch_desc /
qf_decode_batch_desc, k drawn per generation).
"""
from __future__ import annotations

import argparse
import json
import math
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

L_JUMBO, RS = 9000, 9008
REP_RS = 9088   # pool-block repair rows (QF_ENCODE_ZERO_TAIL): bit-sliced pass kernels
SHAPES = [(k, int(np.ceil(np.float32(k) * np.float32(ratio))) - k)
          for k, ratio in ((32, 1.15), (48, 1.15), (64, 1.15), (96, 1.15), (128, 1.15), (160, 1.30), (196, 1.30))]


def timed(ctx, fn, reps):
    fn()
    ctx.sync()
    ctx.profile(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    ctx.sync()
    wall = (time.perf_counter() - t0) / reps * 1e3
    kt = {n: (c / reps, ms / reps) for n, (c, ms) in ctx.kernel_times().items()}
    ctx.profile(False)
    return wall, kt


def device_span(ctx, fn, reps):
    """Device span of `reps` back-to-back calls (HIP events on the context's
    stream, torch's current one here, around the calls; no per-kernel events
    in between) and the host time to enqueue them.  Returns (span ms per call,
    host ms per call)."""
    import torch

    fn()
    ctx.sync()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    host = (time.perf_counter() - t0) / reps * 1e3
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps, host


def mixed_leg(qf, ctx, nbytes: float, reps: int, seed: int = 5) -> dict:
    """One heterogeneous batch (qf_encode_batch_desc / qf_decode_batch_desc):
    k drawn per generation from the C5 shapes, jumbo rows, 20 % source loss,
    encoded in one call and decoded in one call.  Every generation's
    recovered rows are compared with its erased sources (round trip; the
    oracle comparison is tests/test_gpu_desc.py)."""
    import torch

    rng = np.random.default_rng(seed)
    mean_k = float(np.mean([k for k, _ in SHAPES]))
    G = max(len(SHAPES), int(nbytes // (mean_k * L_JUMBO)))
    kind = rng.integers(0, len(SHAPES), G)
    ks = np.array([SHAPES[i][0] for i in kind])
    rs = np.array([SHAPES[i][1] for i in kind])
    es = np.minimum(rs, np.maximum(1, np.round(0.2 * ks))).astype(np.int64)
    src_row0 = np.concatenate([[0], np.cumsum(ks)[:-1]])          # first source row of each generation
    rep_row0 = np.concatenate([[0], np.cumsum(rs)[:-1]])
    nrows = ks - es + rs
    row0 = np.concatenate([[0], np.cumsum(nrows)[:-1]])
    rec_row0 = np.concatenate([[0], np.cumsum(es)[:-1]])
    src = torch.randint(0, 256, (int(ks.sum()) * RS,), dtype=torch.uint8, device="cuda")
    rep = torch.empty(int(rs.sum()) * REP_RS, dtype=torch.uint8, device="cuda")
    # descriptor arrays built once, outside every timed call (VERDICT r04 missing 3)
    gdesc = qf.pack_gen_descs([dict(k=int(ks[g]), r=int(rs[g]), L=L_JUMBO, flags=1,
                                    src_offset=int(src_row0[g]) * RS, src_row_stride=RS,
                                    rep_offset=int(rep_row0[g]) * REP_RS, rep_row_stride=REP_RS) for g in range(G)])

    def enc():
        qf.encode_batch_desc(src, rep, gdesc, ctx=ctx)

    wall_e, kt_e = timed(ctx, enc, reps)
    span_e, host_e = device_span(ctx, enc, reps)
    # received rows: survivors in source order, then every repair; the first
    # k rows are accepted (decoder.rs:679), so the first e repairs decode
    ridx, s_from, s_to, r_from, r_to, lost_src, lost_rec = [], [], [], [], [], [], []
    for g in range(G):
        k, r, e = int(ks[g]), int(rs[g]), int(es[g])
        E = np.sort(rng.choice(k, e, replace=False))
        keep = np.setdiff1d(np.arange(k), E)
        ridx.append(np.concatenate([keep, k + np.arange(r)]).astype(np.uint16))
        s_from.append(src_row0[g] + keep)
        s_to.append(row0[g] + np.arange(k - e))
        r_from.append(rep_row0[g] + np.arange(r))
        r_to.append(row0[g] + k - e + np.arange(r))
        lost_src.append(src_row0[g] + E)
        lost_rec.append(rec_row0[g] + np.arange(e))
    cat = lambda xs: torch.from_numpy(np.concatenate(xs).astype(np.int64)).cuda()  # noqa: E731
    src2 = src.view(-1, RS)
    rep2 = rep.view(-1, REP_RS)[:, :RS]
    rows = torch.empty((int(nrows.sum()), RS), dtype=torch.uint8, device="cuda")
    rows[cat(s_to)] = src2[cat(s_from)]
    rows[cat(r_to)] = rep2[cat(r_from)]
    t_idx = torch.from_numpy(np.concatenate(ridx).view(np.int16)).cuda()
    rec = torch.empty((int(es.sum()), RS), dtype=torch.uint8, device="cuda")
    rec_index = torch.empty(int(rs.sum()), dtype=torch.int16, device="cuda")   # min(k, r) = r entries each
    n_rec = torch.empty(G, dtype=torch.int32, device="cuda")
    status = torch.empty(G, dtype=torch.int32, device="cuda")
    ddesc = qf.pack_dec_descs([dict(k=int(ks[g]), r=int(rs[g]), L=L_JUMBO, n_rows=int(nrows[g]),
                                    rows_offset=int(row0[g]) * RS, row_stride=RS, row_index_offset=int(row0[g]),
                                    rec_offset=int(rec_row0[g]) * RS, rec_row_stride=RS,
                                    rec_index_offset=int(rep_row0[g])) for g in range(G)])

    def dec():
        qf.decode_batch_desc(rows.view(-1), t_idx, rec.view(-1), rec_index, n_rec, status, ddesc, ctx=ctx)

    rec.zero_()
    wall_d, kt_d = timed(ctx, dec, reps)
    span_d, host_d = device_span(ctx, dec, reps)
    ok = bool((status == 0).all().item() and torch.equal(n_rec.cpu(), torch.from_numpy(es.astype(np.int32))))
    ok = ok and torch.equal(rec[:, :L_JUMBO], src2[cat(lost_src)][:, :L_JUMBO])
    kms_e = sum(ms for _, ms in kt_e.values())
    kms_d = sum(ms for _, ms in kt_d.values())
    enc_b = float(((ks + rs) * L_JUMBO).sum())
    dec_b = float(((ks + es) * L_JUMBO).sum())
    return {"G": G, "shapes": {f"k{k}_r{r}": int((kind == i).sum()) for i, (k, r) in enumerate(SHAPES)},
            "round_trip_ok": ok,
            "bytes_rule": "encode (k + r) L, decode (k + e) L per generation; span = HIP events around the call "
                          "(descriptor arrays prebuilt), kernel = sum of the per-kernel HIP events",
            "encode": {"span_ms": round(span_e, 4), "kernel_ms": round(kms_e, 4), "host_call_ms": round(host_e, 4),
                       "span_gibps": round(enc_b / (span_e / 1e3) / 2**30, 1),
                       "kernel_gibps": round(enc_b / (kms_e / 1e3) / 2**30, 1),
                       "span_over_kernel": round(span_e / kms_e, 3),
                       "wall_ms_profiled": round(wall_e, 3), "kernels": kt_e,
                       "GiBps_alg": round(enc_b / (kms_e / 1e3) / 2**30, 1)},
            "decode": {"span_ms": round(span_d, 4), "kernel_ms": round(kms_d, 4), "host_call_ms": round(host_d, 4),
                       "span_gibps": round(dec_b / (span_d / 1e3) / 2**30, 1),
                       "kernel_gibps": round(dec_b / (kms_d / 1e3) / 2**30, 1),
                       "span_over_kernel": round(span_d / kms_d, 3),
                       "wall_ms_profiled": round(wall_d, 3), "kernels": kt_d,
                       "GiBps_alg": round(dec_b / (kms_d / 1e3) / 2**30, 1)}}


# SQ counters of the sliding-window launches (tools/gpu.sh c5sq: rocprofv3
# --pmc over `--modes sliding` of every shape at the G below), keyed by
# kernel name and G, each with the code hash of the kernel it measured
C5_SQ = REPO / "profiles" / "c5_sq_counters.json"
# residency: at least this many generations per leg, so every launch runs
# several rounds of workgroups (>= 4 per CU for the one-wave-per-item
# kernels: G x 568 units / 128 per item / 4 items per workgroup >= 1,024)
G_MIN = 1024


def _valu_info(kt: dict, G: int, L: int, ms: float, mode: str = "block") -> dict | None:
    """VALU issue fraction of the generated encode kernels of a launch set,
    against the kernels' measured time, at 2 cycles per wave64 instruction on
    1,024 SIMDs at 2.4 GHz (MI355X_MICROARCH.md).  The instruction count is
    SQ_INSTS_VALU of a counter pass of the same launches (C5_SQ) where one
    exists for this mode, kernel, G and code hash; otherwise the static model
    (bs_codegen.valu_per_item x items), labelled as such.  None when a kernel
    of the set is not a generated one."""
    from quicfuscate_amd import bs_codegen as bs
    from quicfuscate_amd.build_lib import kernel_specs

    specs = {sp.name: sp for sp in kernel_specs() if sp.mode == "enc"}
    try:
        sq = json.loads(C5_SQ.read_text())
        hashes = json.loads((REPO / "quicfuscate_amd" / "lib" / "kernel_hashes.json").read_text())
    except Exception:
        sq, hashes = {}, {}
    Lv = bs.padded_units(L)
    items = -(-G * Lv // 128)
    instr, counted, cycles = 0, True, 0.0
    for name, (cnt, _) in kt.items():
        sp = specs.get(name)
        if sp is None:
            return None
        ent = sq.get(f"{mode}/{name}/G{G}")
        if ent and ent.get("code_sha16") == hashes.get(name):
            instr += cnt * ent["SQ_INSTS_VALU"]
            cycles += cnt * ent.get("SQ_BUSY_CYCLES", 0.0)
        else:
            counted = False
            instr += cnt * bs.valu_per_item(sp) * items
    issue_ms = instr * 2 / (1024 * 2.4e9) * 1e3
    out = {"valu_instr_per_launch_set": int(instr), "issue_ms": round(issue_ms, 4),
           "frac": round(issue_ms / ms, 4) if ms else None,
           "source": "counters" if counted else "model",
           "model": ("SQ_INSTS_VALU of the same launches (profiles/c5_sq_counters.json, code hash checked)"
                     if counted else "static VALU count per item (bs_codegen.valu_per_item) x items")
           + ", 2 cyc per wave64 instr, 1,024 SIMDs at 2.4 GHz"}
    if counted and cycles:
        out["sq_busy_cycles"] = int(cycles)
    return out


def shape_leg(qf, ctx, k: int, r: int, nbytes: float, reps: int, modes=("block", "sliding"),
              exact_rows: bool = False, verify: bool = True) -> dict:
    """One C5 (k, r) at L = 9,000: block encode ((k + r) L per generation),
    block decode at 20 % source loss ((k + e) L), sliding encode (one window per
    source packet, generation stride = row stride; SURVEY 8(d): (1 + r) L per
    window, compute-bound by construction: its VALU fraction is the roof that
    matters).  Every decode generation's recovered rows are checked against its
    erased sources on the device, and a sample of sliding windows against the
    block encode of the same windows."""
    import torch

    res = {}
    G = max(G_MIN, int(nbytes // (k * L_JUMBO)))
    drs = RS if exact_rows else REP_RS
    for mode in modes:
        if mode == "block":
            src = torch.randint(0, 256, (G * k * RS,), dtype=torch.uint8, device="cuda")
            gs = k * RS
        else:
            src = torch.randint(0, 256, ((G + k - 1) * RS,), dtype=torch.uint8, device="cuda")
            gs = RS
        rep = torch.empty(G * r * drs, dtype=torch.uint8, device="cuda")

        def enc():
            qf.encode_batch(src, rep, k, r, L_JUMBO, src_row_stride=RS, src_gen_stride=gs, rep_row_stride=drs,
                            rep_gen_stride=r * drs, G=G, zero_tail=not exact_rows, ctx=ctx)

        wall, kt = timed(ctx, enc, reps)
        kms = sum(ms for _, ms in kt.values())
        alg = G * ((k + r) if mode == "block" else (1 + r)) * L_JUMBO
        ent = {"G": G, "wall_ms": round(wall, 3), "kernels": kt,
               "algorithmic_bytes": alg, "bytes_rule": "(k + r) L per generation" if mode == "block" else
               "(1 + r) L per window (SURVEY 8(d): one new source row read, r repairs written)",
               "GiBps_alg": round(alg / (kms / 1e3) / 2**30, 1),
               "hbm_frac_of_8TBps": round(alg / (kms / 1e3) / 8e12, 3),
               "valu": _valu_info(kt, G, L_JUMBO, kms, mode)}
        if mode == "sliding" and verify:
            # windows g = 0, G/2, G-1 re-encoded as a block batch
            wins = sorted({0, G // 2, G - 1})
            blk = torch.stack([src.view(-1, RS)[g:g + k] for g in wins]).reshape(-1)
            rb = torch.empty(len(wins) * r * drs, dtype=torch.uint8, device="cuda")
            qf.encode_batch(blk, rb, k, r, L_JUMBO, src_row_stride=RS, src_gen_stride=k * RS, rep_row_stride=drs,
                            rep_gen_stride=r * drs, G=len(wins), zero_tail=not exact_rows, ctx=ctx)
            ctx.sync()
            got = rep.view(G, r, drs)[wins, :, :L_JUMBO]
            ent["verified_windows"] = len(wins)
            ent["verified"] = bool(torch.equal(got, rb.view(len(wins), r, drs)[:, :, :L_JUMBO]))
        res[f"{mode}/encode"] = ent
        if mode == "block":
            # decode at 20 % source loss (first k rows: survivors then repairs)
            e = min(r, max(1, round(0.2 * k)))
            max_rows = k - e + r
            rng = np.random.default_rng(k)
            keys = rng.random((G, k))
            er = np.sort(np.argsort(keys, axis=1)[:, :e], axis=1)
            keep = np.ones((G, k), bool)
            np.put_along_axis(keep, er, False, axis=1)
            ridx = np.zeros((G, max_rows), np.uint16)
            ridx[:, :k - e] = np.nonzero(keep)[1].reshape(G, k - e)
            ridx[:, k - e:] = k + np.arange(r)
            ai = torch.from_numpy(ridx.astype(np.int64)).cuda()
            src3 = src.view(G, k, RS)
            rep3 = rep.view(G, r, drs)[:, :, :RS]
            rows = torch.empty((G, max_rows, RS), dtype=torch.uint8, device="cuda")
            for g0 in range(0, G, 256):
                g1 = min(G, g0 + 256)
                sel = ai[g0:g1]
                gi = torch.arange(g0, g1, device="cuda")[:, None]
                rows[g0:g1] = torch.where((sel < k)[..., None], src3[gi, sel.clamp(max=k - 1)],
                                          rep3[gi, (sel - k).clamp(min=0)])
            t_idx = torch.from_numpy(ridx.view(np.int16).reshape(-1)).cuda()
            rec = torch.empty(G * e * RS, dtype=torch.uint8, device="cuda")
            rec_index = torch.empty(G * min(k, r), dtype=torch.int16, device="cuda")   # min(k, r) per generation
            n_rec = torch.empty(G, dtype=torch.int32, device="cuda")
            status = torch.empty(G, dtype=torch.int32, device="cuda")

            def dec():
                qf.decode_batch(rows.view(-1), t_idx, rec, rec_index, n_rec, status, k, r, L_JUMBO,
                                max_rows=max_rows, row_stride=RS, rows_gen_stride=max_rows * RS,
                                rec_row_stride=RS, rec_gen_stride=e * RS, G=G, ctx=ctx)

            wall, kt = timed(ctx, dec, reps)
            ok = bool((status == 0).all().item() and (n_rec == e).all().item())
            if verify and ok:
                et = torch.from_numpy(er.astype(np.int64)).cuda()
                gi = torch.arange(G, device="cuda")[:, None].expand(-1, e)
                ok = bool(torch.equal(rec.view(G, e, RS)[:, :, :L_JUMBO], src3[gi, et][:, :, :L_JUMBO]))
                ok = ok and bool((rec_index.view(G, min(k, r))[:, :e].long() == et).all().item())
            kms = sum(ms for _, ms in kt.values())
            res["block/decode"] = {"G": G, "erased": e, "wall_ms": round(wall, 3), "kernels": kt,
                                   "GiBps_alg": round(G * (k + e) * L_JUMBO / (kms / 1e3) / 2**30, 1),
                                   "hbm_frac_of_8TBps": round(G * (k + e) * L_JUMBO / (kms / 1e3) / 8e12, 3),
                                   "verified": ok}
            del rows, rec
        del src, rep
        torch.cuda.empty_cache()
    return res


def c5_bench(qf, ctx, mixed_bytes: float = 4e9, shape_bytes: float = 1e9, reps: int = 3, shapes=None,
             modes=("block", "sliding"), mixed: bool = True, exact_rows: bool = False) -> dict:
    """BASELINE configs[4]: the heterogeneous batch of all
    seven shapes (>= 4 GB of source) plus block and sliding per shape.  Used by
    bench.py's `c5` leg and by this tool's command line."""
    out = {"L": L_JUMBO, "row_stride": RS, "repair_row_stride": REP_RS, "loss": 0.2}
    if mixed:
        out["mixed_desc_batch"] = mixed_leg(qf, ctx, mixed_bytes, reps)
    for k, r in (shapes or SHAPES):
        out[f"k{k}_r{r}"] = shape_leg(qf, ctx, k, r, shape_bytes, reps, modes, exact_rows)
    return out


def main():
    from quicfuscate_amd import fec as qf

    ap = argparse.ArgumentParser()
    ap.add_argument("--bytes", type=float, default=1e9, help="source bytes per shape and mode")
    ap.add_argument("--mixed-bytes", type=float, default=4e9, help="source bytes of the heterogeneous batch")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default="gpurun_out/c5_bench.json")
    ap.add_argument("--exact-rows", action="store_true",
                    help="dense repair rows without the zero tail (general v_perm encode kernel)")
    ap.add_argument("--mixed-only", action="store_true", help="only the heterogeneous (desc API) batch")
    ap.add_argument("--shapes", default="", help="k,r[;k,r...]: only these block/sliding shapes, no mixed batch")
    ap.add_argument("--modes", default="block,sliding")
    a = ap.parse_args()
    ctx = qf.default_context()
    shapes = SHAPES
    if a.shapes:
        shapes = [tuple(int(x) for x in s.split(",")) for s in a.shapes.split(";")]
    res = c5_bench(qf, ctx, a.mixed_bytes, a.bytes, a.reps, [] if a.mixed_only else shapes,
                   tuple(a.modes.split(",")), mixed=not a.shapes, exact_rows=a.exact_rows)
    for key, v in res.items():
        if key.startswith("k"):
            print(key, {m: (e["GiBps_alg"], e.get("hbm_frac_of_8TBps"), (e.get("valu") or {}).get("frac"))
                        for m, e in v.items()}, flush=True)
    Path(a.out).parent.mkdir(exist_ok=True)
    Path(a.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
