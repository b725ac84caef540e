#!/usr/bin/env python3
"""BASELINE C5 throughput on the MI355X (diagnostic beside bench.py): the
adaptive sliding-window shapes of SURVEY 8(d) -- k 32..196, r = ceil(k*ratio)-k,
9000-byte jumbo payloads -- in block mode (independent generations) and
sliding mode (one window per source packet: generation stride = row stride),
encode and decode at 20 % source loss, device-resident, HIP-event kernel
times.  Algorithmic bytes: encode (k + r) L per generation, decode (k + e) L.

    python tools/bench_c5.py [--bytes 2e9] [--out gpurun_out/c5_bench.json] [--mixed-only]

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
    gdesc = [dict(k=int(ks[g]), r=int(rs[g]), L=L_JUMBO, flags=1, src_offset=int(src_row0[g]) * RS, src_row_stride=RS,
                  rep_offset=int(rep_row0[g]) * REP_RS, rep_row_stride=REP_RS) for g in range(G)]

    def enc():
        qf.encode_batch_desc(src, rep, gdesc)

    wall_e, kt_e = timed(ctx, enc, reps)
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
    ddesc = [dict(k=int(ks[g]), r=int(rs[g]), L=L_JUMBO, n_rows=int(nrows[g]), rows_offset=int(row0[g]) * RS,
                  row_stride=RS, row_index_offset=int(row0[g]), rec_offset=int(rec_row0[g]) * RS, rec_row_stride=RS,
                  rec_index_offset=int(rep_row0[g])) for g in range(G)]

    def dec():
        qf.decode_batch_desc(rows.view(-1), t_idx, rec.view(-1), rec_index, n_rec, status, ddesc)

    wall_d, kt_d = timed(ctx, dec, reps)
    ok = bool((status == 0).all().item() and torch.equal(n_rec.cpu(), torch.from_numpy(es.astype(np.int32))))
    ok = ok and torch.equal(rec[:, :L_JUMBO], src2[cat(lost_src)][:, :L_JUMBO])
    kms_e = sum(ms for _, ms in kt_e.values())
    kms_d = sum(ms for _, ms in kt_d.values())
    enc_b = float(((ks + rs) * L_JUMBO).sum())
    dec_b = float(((ks + es) * L_JUMBO).sum())
    return {"G": G, "shapes": {f"k{k}_r{r}": int((kind == i).sum()) for i, (k, r) in enumerate(SHAPES)},
            "round_trip_ok": ok,
            "encode": {"wall_ms": round(wall_e, 3), "kernels": kt_e,
                       "GiBps_alg": round(enc_b / (kms_e / 1e3) / 2**30, 1),
                       "GiBps_wall": round(enc_b / (wall_e / 1e3) / 2**30, 1)},
            "decode": {"wall_ms": round(wall_d, 3), "kernels": kt_d,
                       "GiBps_alg": round(dec_b / (kms_d / 1e3) / 2**30, 1),
                       "GiBps_wall": round(dec_b / (wall_d / 1e3) / 2**30, 1)}}


def main():
    import torch

    from quicfuscate_amd import fec as qf

    ap = argparse.ArgumentParser()
    ap.add_argument("--bytes", type=float, default=2e9, help="source bytes per shape and mode")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default="gpurun_out/c5_bench.json")
    ap.add_argument("--exact-rows", action="store_true",
                    help="dense repair rows without the zero tail (general v_perm encode kernel)")
    ap.add_argument("--mixed-only", action="store_true", help="only the heterogeneous (desc API) batch")
    ap.add_argument("--shapes", default="", help="k,r[;k,r...]: only these block/sliding shapes, no mixed batch")
    ap.add_argument("--modes", default="block,sliding")
    a = ap.parse_args()
    ctx = qf.default_context()
    res = {}
    shapes = SHAPES
    if a.shapes:
        shapes = [tuple(int(x) for x in s.split(",")) for s in a.shapes.split(";")]
    else:
        res["mixed_desc_batch"] = mixed_leg(qf, ctx, a.bytes, a.reps)
        print("mixed", {k: v for k, v in res["mixed_desc_batch"].items() if k in ("G", "round_trip_ok")},
              res["mixed_desc_batch"]["encode"]["GiBps_alg"], res["mixed_desc_batch"]["decode"]["GiBps_alg"],
              flush=True)
    for k, r in ([] if a.mixed_only else shapes):
        G = max(1, int(a.bytes // (k * L_JUMBO)))
        for mode in a.modes.split(","):
            if mode == "block":
                src = torch.randint(0, 256, (G * k * RS,), dtype=torch.uint8, device="cuda")
                gs = k * RS
            else:
                src = torch.randint(0, 256, ((G + k - 1) * RS,), dtype=torch.uint8, device="cuda")
                gs = RS
            drs = RS if a.exact_rows else REP_RS
            rep = torch.empty(G * r * drs, dtype=torch.uint8, device="cuda")

            def enc():
                qf.encode_batch(src, rep, k, r, L_JUMBO, src_row_stride=RS, src_gen_stride=gs, rep_row_stride=drs,
                                rep_gen_stride=r * drs, G=G, zero_tail=not a.exact_rows)

            wall, kt = timed(ctx, enc, a.reps)
            kms = sum(ms for _, ms in kt.values())
            res[f"k{k}_r{r}/{mode}/encode"] = {"G": G, "wall_ms": round(wall, 3), "kernels": kt,
                                               "GiBps_alg": round(G * (k + r) * L_JUMBO / (kms / 1e3) / 2**30, 1),
                                               "frac_of_8TBps": round(G * (k + r) * L_JUMBO / (kms / 1e3) / 8e12, 3)}
            if mode == "block":
                # decode at 20 % source loss (first k rows: survivors then repairs)
                e = min(r, max(1, round(0.2 * k)))
                max_rows = k - e + r
                rng = np.random.default_rng(k)
                ridx = np.zeros((G, max_rows), np.uint16)
                for g in range(G):
                    E = set(rng.choice(k, e, replace=False).tolist())
                    ridx[g] = [i for i in range(k) if i not in E] + [k + j for j in range(r)]
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
                                    rec_row_stride=RS, rec_gen_stride=e * RS, G=G)

                wall, kt = timed(ctx, dec, a.reps)
                if not ((status == 0).all().item() and (n_rec == e).all().item()):
                    st_np, nr_np = status.cpu().numpy(), n_rec.cpu().numpy()
                    raise AssertionError(f"k={k} r={r} G={G}: statuses {np.unique(st_np, return_counts=True)}, "
                                         f"n_rec {np.unique(nr_np, return_counts=True)} (expected {e})")
                g = G - 1
                E = sorted(set(range(k)) - set(int(x) for x in ridx[g] if x < k))
                assert torch.equal(rec.view(G, e, RS)[g, :, :L_JUMBO], src3[g, E, :L_JUMBO])
                kms = sum(ms for _, ms in kt.values())
                res[f"k{k}_r{r}/block/decode"] = {"G": G, "erased": e, "wall_ms": round(wall, 3), "kernels": kt,
                                                   "GiBps_alg": round(G * (k + e) * L_JUMBO / (kms / 1e3) / 2**30, 1)}
                del rows, rec
            del src, rep
            torch.cuda.empty_cache()
        print(k, r, {kk: v["GiBps_alg"] for kk, v in res.items() if kk.startswith(f"k{k}_")}, flush=True)
    Path(a.out).parent.mkdir(exist_ok=True)
    Path(a.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
