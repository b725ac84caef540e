#!/usr/bin/env python3
"""VGPR operand banks and the issue rate of 2- and 3-source VALU ops on gfx950
(diagnostic).  Hand-written assembly loops (assembled like the generated
kernels, build_lib.assemble): 8 independent destination chains, each op
reading its destination and one or two source VGPRs whose register numbers
are chosen so that the operands fall in the same or in different banks
(bank = register number mod 4, the GCN rule this measures).

    python tools/ubench_banks.py build      # here
    python tools/ubench_banks.py run        # GPU box: wave64 ops per SIMD per ns, 1 and 2 waves per SIMD
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
ITERS = 4096
OPS = 64


def _ops(kind: str) -> list[str]:
    """64 ops over 8 chains.  dest v(16 + 4 c) sits in bank 0 for every chain c;
    sources: bank 0 (same as dest) = v(48 + 4 j), bank 1 = v(49 + 4 j), bank 2 = v(50 + 4 j)."""
    out = []
    for n in range(OPS):
        c = n % 8
        d = 16 + 4 * c
        j = n % 4
        b0, b1, b2 = 48 + 4 * j, 49 + 4 * j, 50 + 4 * j
        if kind == "xor_diff":
            out.append(f"v_xor_b32_e32 v{d}, v{b1}, v{d}")
        elif kind == "xor_same":
            out.append(f"v_xor_b32_e32 v{d}, v{b0}, v{d}")
        elif kind == "bop_diff":      # d, b1, b2: three banks
            out.append(f"v_bitop3_b32 v{d}, v{d}, v{b1}, v{b2} bitop3:0x96")
        elif kind == "bop_2same":     # b1 twice-bank: two sources in bank 1
            out.append(f"v_bitop3_b32 v{d}, v{d}, v{b1}, v{49 + 4 * ((j + 1) % 4)} bitop3:0x96")
        elif kind == "bop_3same":     # all three in bank 0
            out.append(f"v_bitop3_b32 v{d}, v{d}, v{b0}, v{48 + 4 * ((j + 1) % 4)} bitop3:0x96")
        elif kind == "bop_dsame":     # a source in the destination's bank
            out.append(f"v_bitop3_b32 v{d}, v{d}, v{b0}, v{b1} bitop3:0x96")
        elif kind == "bsel_s_diff":   # SGPR mask, two VGPRs in different banks
            out.append(f"v_bitop3_b32 v{d}, s40, v{d}, v{b1} bitop3:0xca")
        elif kind == "perm_diff":
            out.append(f"v_perm_b32 v{d}, v{b1}, v{b2}, v{d}")
        elif kind == "perm_same":
            out.append(f"v_perm_b32 v{d}, v{b0}, v{48 + 4 * ((j + 1) % 4)}, v{d}")
        else:
            raise ValueError(kind)
    return out


KINDS = ["xor_diff", "xor_same", "bop_diff", "bop_2same", "bop_3same", "bop_dsame", "bsel_s_diff", "perm_diff",
         "perm_same"]
# straight-line code (no loop): LINE x 64 ops unrolled, ITERS // LINE passes of
# an outer loop -- the same op count as the looped kinds, but the code of one
# pass is LINE times larger (instruction fetch beyond the instruction cache)
# (s_cbranch reaches +-128 KiB: at most ~240 x 64 eight-byte ops per pass)
LINES = {"bop_diff_line16": ("bop_diff", 16), "bop_diff_line64": ("bop_diff", 64),
         "bop_diff_line128": ("bop_diff", 128), "bop_diff_line240": ("bop_diff", 240),
         "xor_diff_line240": ("xor_diff", 240)}
KINDS += list(LINES)
# the same straight-line loop copied to NB addresses: wave w of workgroup g runs
# copy (w + 4 (g & 1)) % NB, so the CU's waves fetch NB different code streams
# (the merged C5 encode runs 4 pass bodies of ~200 KB on every CU)
DISTINCT = {"bop_diff_line16_d4": ("bop_diff", 16, 4), "bop_diff_line64_d4": ("bop_diff", 64, 4),
            "bop_diff_line240_d4": ("bop_diff", 240, 4), "bop_diff_line64_d8": ("bop_diff", 64, 8),
            "bop_diff_line240_d8": ("bop_diff", 240, 8), "xor_diff_line240_d4": ("xor_diff", 240, 4)}
KINDS += list(DISTINCT)


class _Spec:
    def __init__(self, name):
        self.name = name
        self.next_free_vgpr = 72
        self.next_free_sgpr = 48
        self.kernarg_bytes = 24
        self.lds_bytes = 0
        self.waves = 4


def _asm(kind: str) -> tuple[str, str]:
    from quicfuscate_amd import bs_codegen as bs

    name = f"ub_{kind}"
    base, line, nb = DISTINCT.get(kind, LINES.get(kind, (kind, 1)) + (1,))
    body = [f"s_mov_b32 s20, {max(1, ITERS // line)}", "s_mov_b32 s40, 0x0f0f0f0f"]
    for r in range(16, 72):
        body.append(f"v_mov_b32_e32 v{r}, {r * 2654435761 & 0xFFFF}")
    if nb > 1:
        # copy index (wave + 4 (workgroup & 1)) % nb; far jumps (copies > 128 KiB apart)
        body += ["v_lshrrev_b32_e32 v1, 6, v0", "v_readfirstlane_b32 s21, v1", "s_and_b32 s22, s2, 1",
                 "s_lshl_b32 s22, s22, 2", "s_add_u32 s21, s21, s22", f"s_and_b32 s21, s21, {nb - 1}"]
        for c in range(1, nb):
            body += [f"s_cmp_lg_u32 s21, {c}", f"s_cbranch_scc1 .Lnc{c}", "s_getpc_b64 s[24:25]", f".Lfar{c}:",
                     f"s_add_u32 s24, s24, (.Lcopy{c}-.Lfar{c})&4294967295",
                     f"s_addc_u32 s25, s25, (.Lcopy{c}-.Lfar{c})>>32", "s_setpc_b64 s[24:25]", f".Lnc{c}:"]
    for c in range(nb):
        body.append(f".Lcopy{c}:")
        body.append(f".Lloop{c}:")
        for _ in range(line):
            body += _ops(base)
        body += ["s_sub_u32 s20, s20, 1", "s_cmp_lg_u32 s20, 0", f"s_cbranch_scc1 .Lloop{c}", "s_endpgm"]

    class Op:
        def __init__(self, s):
            self.s, self.name, self.args = s, ("label" if s.endswith(":") else "raw"), (s[:-1],) if s.endswith(":") else ()

        def asm(self):
            return self.s
    return name, bs.emit_asm(_Spec(name), [Op(s) for s in body])


def build():
    from quicfuscate_amd.build_lib import assemble

    OUT.mkdir(parents=True, exist_ok=True)
    man = []
    for kind in KINDS:
        name, text = _asm(kind)
        h = assemble(name, text, OUT)
        man.append({"kind": kind, "hsaco": h.name, "symbol": name})
    (OUT / "ub_banks.json").write_text(json.dumps(man, indent=1))


def run():
    import torch

    hip = ctypes.CDLL(str(Path(torch.__file__).parent / "lib" / "libamdhip64.so"))
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    stream = torch.cuda.current_stream()
    res = {}
    kbuf = ctypes.create_string_buffer(24)
    size = ctypes.c_size_t(24)
    extra = (ctypes.c_void_p * 5)(1, ctypes.cast(kbuf, ctypes.c_void_p), 2,
                                 ctypes.cast(ctypes.pointer(size), ctypes.c_void_p), 3)
    for m in json.loads((OUT / "ub_banks.json").read_text()):
        mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
        data = (OUT / m["hsaco"]).read_bytes()
        buf = ctypes.create_string_buffer(data, len(data))
        assert hip.hipModuleLoadData(ctypes.byref(mod), buf) == 0
        assert hip.hipModuleGetFunction(ctypes.byref(fn), mod, m["symbol"].encode()) == 0
        for w in (1, 2):
            blocks = cus * w

            def launch():
                assert hip.hipModuleLaunchKernel(fn, blocks, 1, 1, 256, 1, 1, 0, ctypes.c_void_p(stream.cuda_stream),
                                                 None, extra) == 0
            launch()
            torch.cuda.synchronize()
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record(stream)
            for _ in range(5):
                launch()
            t1.record(stream)
            torch.cuda.synchronize()
            ms = t0.elapsed_time(t1) / 5
            base, line, _ = DISTINCT.get(m["kind"], LINES.get(m["kind"], (m["kind"], 1)) + (1,))
            per_simd = blocks * 4 * OPS * line * max(1, ITERS // line) / (cus * 4) / (ms * 1e6)
            res[f"{m['kind']}_w{w}"] = round(per_simd, 4)
            print(m["kind"], w, res[f"{m['kind']}_w{w}"], flush=True)
        hip.hipModuleUnload(mod)
    return res


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["build", "run"])
    ap.add_argument("--out", default="gpurun_out/ub_banks.json")
    a = ap.parse_args()
    if a.cmd == "build":
        build()
    else:
        r = run()
        Path(a.out).parent.mkdir(exist_ok=True)
        Path(a.out).write_text(json.dumps({"unit": "wave64 ops per SIMD per ns", "results": r}, indent=1))
