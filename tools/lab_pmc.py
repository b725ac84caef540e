#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE per lab kernel (tools/bs_lab.py, tools/dec_lab.py
builds: every variant has its own symbol lab_<name>) against the bytes the
variant is known to move.

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/lf -- python3 tools/bs_lab.py run --reps 3
    rocprofv3 --pmc WRITE_SIZE -d gpurun_out/lw -- python3 tools/bs_lab.py run --reps 3
    python3 tools/lab_pmc.py gpurun_out/lf gpurun_out/lw --G 65536 --out profiles/r04_traffic.json

Known bytes (encode lab): reads G k L of source (a `nostore` variant writes
nothing), writes G r 16 Lv (zero-tail rows).  FETCH_SIZE is doubled (the
guide's gfx950 correction for wide streaming reads); the L:1024 read-only
variants calibrate that factor on this very access pattern (line-aligned
rows: no line is shared by two rows or two items).
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "tools"))
sys.path.insert(0, str(REPO))

from pmc_traffic import per_dispatch  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--G", type=int, default=65536)
    ap.add_argument("--manifest", default=str(REPO / "tools" / "lab_build" / "manifest.json"))
    ap.add_argument("--out", default="")
    ap.add_argument("--command", default="")
    ap.add_argument("--dec", action="store_true", help="decode lab (dec_manifest.json): k = 64 rows read, e = 13 written")
    a = ap.parse_args()
    from quicfuscate_amd import bs_codegen as bs

    fetch = per_dispatch(Path(a.fetch_dir), "FETCH_SIZE")
    write = per_dispatch(Path(a.write_dir), "WRITE_SIZE")
    mpath = Path(a.manifest)
    if a.dec and mpath.name == "manifest.json":
        mpath = mpath.with_name("dec_manifest.json")
    man = {m["symbol"]: m for m in json.loads(mpath.read_text())}
    out = {"_note": "FETCH_SIZE(KiB)*1024*2 and WRITE_SIZE(KiB)*1024, median over dispatches, per lab kernel; "
                    "known = the bytes the variant must move (source reads G k L; zero-tail repair writes G r 16 Lv)",
           "_command": a.command, "G": a.G}
    for sym, m in man.items():
        f = [v for n, vs in fetch.items() if sym in n for v in vs]
        w = [v for n, vs in write.items() if sym in n for v in vs]
        if not f:
            continue
        if a.dec:   # C3 shape: 64 received rows read (the 13 zero rows hit L2), 13 rows written
            L = 1200
            known_r = a.G * 64 * L
            known_w = 0 if "nostore" in m["flags"] else a.G * 13 * L
        else:
            k, r, L = m["k"], m["r"], m["L"]
            Lv = bs.padded_units(L)
            known_r = a.G * k * L
            known_w = 0 if "nostore" in m["flags"] else a.G * r * 16 * Lv
        fb = statistics.median(f) * 1024 * 2
        wb = statistics.median(w) * 1024 if w else None
        out[m["name"]] = {"flags": m["flags"], "kw": m.get("kw"), "L": L, "known_read_bytes": known_r, "fetch_bytes_x2": int(fb),
                          "read_ratio": round(fb / known_r, 4), "known_write_bytes": known_w,
                          "write_bytes": None if wb is None else int(wb),
                          "write_ratio": None if not (wb and known_w) else round(wb / known_w, 4),
                          "dispatches": len(f)}
        print(m["name"], out[m["name"]])
    if a.out:
        Path(a.out).write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
