"""Generator of the bit-sliced Cauchy encode kernel for gfx950 (assembly).

Why: on gfx950 v_perm_b32 / v_bitop3_b32 issue at about half rate while
2-operand v_xor_b32 / v_and_b32 / shifts are full rate (tools/ubench.hip,
profiles/r01_ubench_valu_rates.json).  The reference's repair coefficients
are a fixed Cauchy matrix per (k, r) (decoder.rs:280-298), so multiplication
by each coefficient can be specialised into straight-line XOR code over
bit-planes:

  * a lane owns a 32-byte chunk of a row (8 dwords);
  * a 3-stage delta-swap network transposes the chunk into 8 bit-planes
    (plane a = bit a of all 32 bytes);
  * c * x over GF(2^8) is the GF(2)-linear map M_c (column a = c * 2^a), so
    output plane b = XOR_a M_c[b][a] * plane_a;
  * the 15 nonzero XOR combinations of planes 0..3 (L[v]) and of planes 4..7
    (H[v]) are formed once per row, so every output plane of every
    coefficient is acc ^= L[lo] ^= H[hi]: ~15 full-rate v_xor_b32 per
    coefficient for 32 bytes x 64 lanes = 2048 byte multiply-adds;
  * the same delta-swap network (an involution) turns the accumulated
    planes back into bytes.

The row loop is fully unrolled (coefficients are immediates of the code, ~100
KB of straight-line code; tools/ubench_icache.hip shows no instruction-cache
penalty at that size).  Rows stream through a ring of PD+1 register buffers
with explicit global_load_dwordx4 / s_waitcnt vmcnt(N).

The generator builds a small IR that is (1) emitted as assembly and (2)
executed by `Emulator` (64 lanes, numpy) in the CPU test-suite, which checks
results against the oracle, every memory access against the buffer bounds
and every register read against outstanding loads (a missing vmcnt wait).
"""
from __future__ import annotations

import dataclasses
import functools
from typing import Optional

import numpy as np

MASK32 = 0xFFFFFFFF

# --------------------------------------------------------------------------
# GF(2^8) (poly 0x11D, generator 2) -- gf_tables.rs:384-408
# --------------------------------------------------------------------------
_EXP = [0] * 512
_LOG = [0] * 256
_x = 1
for _i in range(255):
    _EXP[_i] = _EXP[_i + 255] = _x
    _LOG[_x] = _i
    _x <<= 1
    if _x >= 256:
        _x ^= 0x11D


def gf_mul(a: int, b: int) -> int:
    return 0 if a == 0 or b == 0 else _EXP[_LOG[a] + _LOG[b]]


def gf_inv(a: int) -> int:
    if a == 0:
        raise ZeroDivisionError
    return _EXP[255 - _LOG[a]]


def cauchy(k: int, r: int) -> list[list[int]]:
    """decoder.rs:280-298: C[j][i] = inv((i as u8) ^ ((k + j) as u8))."""
    return [[gf_inv((i & 0xFF) ^ ((k + j) & 0xFF)) for i in range(k)] for j in range(r)]


def mul_matrix_rows(c: int) -> list[int]:
    """Row b of M_c as a bitmask over input planes a (bit a set iff
    bit b of c * 2^a is set)."""
    cols = [gf_mul(c, 1 << a) for a in range(8)]
    return [sum(((cols[a] >> b) & 1) << a for a in range(8)) for b in range(8)]


# --------------------------------------------------------------------------
# IR
# --------------------------------------------------------------------------
@dataclasses.dataclass
class Op:
    name: str
    args: tuple

    def asm(self) -> str:
        f = _ASM.get(self.name)
        return f(*self.args) if f else f"{self.name} " + ", ".join(map(str, self.args))


def V(i):
    return f"v{i}"


def VP(i):
    return f"v[{i}:{i + 1}]"


def VQ(i):
    return f"v[{i}:{i + 3}]"


def SP(i):
    return f"s[{i}:{i + 1}]"


_ASM = {
    "label": lambda n: f"{n}:",
    "v_xor": lambda d, a, b: f"v_xor_b32_e32 {V(d)}, {V(a)}, {V(b)}",
    "v_mov": lambda d, a: f"v_mov_b32_e32 {V(d)}, {V(a)}",
    "v_xor3": lambda d, a, b, c: f"v_bitop3_b32 {V(d)}, {V(a)}, {V(b)}, {V(c)} bitop3:0x96",
    # d = (s[m] & a) | (~s[m] & b): bit select (truth table index s0*4 + s1*2 + s2)
    "v_bitsel_s": lambda d, m, a, b: f"v_bitop3_b32 {V(d)}, s{m}, {V(a)}, {V(b)} bitop3:0xca",
    # the same bit-select with the mask in a VGPR: v_bitop3 with an SGPR operand
    # issues at half the rate of an all-VGPR one (tools/ubench_idx.py)
    "v_bitsel_v": lambda d, m, a, b: f"v_bitop3_b32 {V(d)}, {V(m)}, {V(a)}, {V(b)} bitop3:0xca",
    "v_movk": lambda d, k: f"v_mov_b32_e32 {V(d)}, {k}",
    "v_andk": lambda d, k, a: f"v_and_b32_e32 {V(d)}, 0x{k:08x}, {V(a)}",
    "v_lshr": lambda d, s, a: f"v_lshrrev_b32_e32 {V(d)}, {s}, {V(a)}",
    "v_lshl": lambda d, s, a: f"v_lshlrev_b32_e32 {V(d)}, {s}, {V(a)}",
    "v_lshl64": lambda d, s, a: f"v_lshlrev_b64 {VP(d)}, {s}, {VP(a)}",
    "v_lshr64": lambda d, s, a: f"v_lshrrev_b64 {VP(d)}, {s}, {VP(a)}",
    "v_lshr_s": lambda d, s, a: f"v_lshrrev_b32_e64 {V(d)}, s{s}, {V(a)}",
    "v_addk": lambda d, k, a: f"v_add_u32_e32 {V(d)}, {k}, {V(a)}",
    "v_add_s": lambda d, s_, a: f"v_add_u32_e32 {V(d)}, s{s_}, {V(a)}",
    "v_sub": lambda d, a, b: f"v_sub_u32_e32 {V(d)}, {V(a)}, {V(b)}",
    "v_lshl_add_s": lambda d, s, sh, a: f"v_lshl_add_u32 {V(d)}, s{s}, {sh}, {V(a)}",
    "v_mul_hi_s": lambda d, a, s: f"v_mul_hi_u32 {V(d)}, {V(a)}, s{s}",
    "v_mul_lo_s": lambda d, a, s: f"v_mul_lo_u32 {V(d)}, {V(a)}, s{s}",
    "v_movs": lambda d, s: f"v_mov_b32_e32 {V(d)}, s{s}",
    "v_mad64_s": lambda d, a, s, c: f"v_mad_u64_u32 {VP(d)}, s[36:37], {V(a)}, s{s}, {VP(c)}",
    "v_mad64_k": lambda d, a, k, c: f"v_mad_u64_u32 {VP(d)}, s[36:37], {V(a)}, {k}, {VP(c)}",
    "v_add64_s": lambda d, a, s: f"v_lshl_add_u64 {VP(d)}, {VP(a)}, 0, {SP(s)}",
    "v_cmp_gt_s": lambda sd, s, a: f"v_cmp_gt_u32_e64 {SP(sd)}, s{s}, {V(a)}",
    "v_cmp_ge_s": lambda sd, s, a: f"v_cmp_ge_u32_e64 {SP(sd)}, s{s}, {V(a)}",
    "v_readfirstlane": lambda s, a: f"v_readfirstlane_b32 s{s}, {V(a)}",
    "v_bfe": lambda d, a, off, w: f"v_bfe_u32 {V(d)}, {V(a)}, {off}, {w}",
    "v_cmp_ne_s": lambda sd, s, a: f"v_cmp_ne_u32_e64 {SP(sd)}, s{s}, {V(a)}",
    "v_cmp_eq_s": lambda sd, s, a: f"v_cmp_eq_u32_e64 {SP(sd)}, s{s}, {V(a)}",
    "v_and_s": lambda d, s, a: f"v_and_b32_e32 {V(d)}, s{s}, {V(a)}",
    "s_cbranch_execz": lambda lbl: f"s_cbranch_execz {lbl}",
    "s_cmp_eq_k_br": lambda s, kk, lbl: f"s_cmp_eq_u32 s{s}, 0x{kk:x}\n\ts_cbranch_scc1 {lbl}",
    "v_cndmask": lambda d, a, b, sm: f"v_cndmask_b32_e64 {V(d)}, {V(a)}, {V(b)}, {SP(sm)}",
    "load16": lambda d, a, off, pol="": f"global_load_dwordx4 {VQ(d)}, {VP(a)}, off"
              + (f" offset:{off}" if off else "") + (f" {pol}" if pol else ""),
    "store16": lambda a, d, off, pol="": f"global_store_dwordx4 {VP(a)}, {VQ(d)}, off"
               + (f" offset:{off}" if off else "") + (f" {pol}" if pol else ""),
    "s_exec": lambda s: "s_mov_b64 exec, -1" if s is None else f"s_mov_b64 exec, {SP(s)}",
    "s_and64": lambda d, a, b: f"s_and_b64 {SP(d)}, {SP(a)}, {SP(b)}",
    "s_andn2_64": lambda d, a, b: f"s_andn2_b64 {SP(d)}, {SP(a)}, {SP(b)}",
    "s_mov": lambda d, a: f"s_mov_b32 s{d}, s{a}",
    "s_movk": lambda d, k: f"s_mov_b32 s{d}, {k}",
    "s_add": lambda d, a, b: f"s_add_u32 s{d}, s{a}, s{b}",
    "s_lshl": lambda d, a, k: f"s_lshl_b32 s{d}, s{a}, {k}",
    "s_lshrk": lambda d, a, k: f"s_lshr_b32 s{d}, s{a}, {k}",
    "s_andk": lambda d, a, k: f"s_and_b32 s{d}, s{a}, {k}",
    "s_mul": lambda d, a, b: f"s_mul_i32 s{d}, s{a}, s{b}",
    "s_mul_k": lambda d, a, kk: f"s_mul_i32 s{d}, s{a}, {kk}",
    "s_m0": lambda a, kk: f"s_add_u32 m0, s{a}, {kk}",
    "load16_lds": lambda a, pol="": f"global_load_lds_dwordx4 {VP(a)}, off" + (f" {pol}" if pol else ""),
    "s_ashr31": lambda d, a: f"s_ashr_i32 s{d}, s{a}, 31",
    "s_min": lambda d, a, b: f"s_min_u32 s{d}, s{a}, s{b}",
    "s_cmp_ge_br": lambda a, b, lbl: f"s_cmp_ge_u32 s{a}, s{b}\n\ts_cbranch_scc1 {lbl}",
    "s_branch": lambda lbl: f"s_branch {lbl}",
    "s_cmp_lt_br": lambda a, b, lbl: f"s_cmp_lt_u32 s{a}, s{b}\n\ts_cbranch_scc1 {lbl}",
    # branch beyond the +-128 KiB of s_branch (the dec kernel is ~200 KiB):
    # pc-relative 64-bit jump through s[66:67]
    "s_far_jump": lambda lbl, n: (f"s_getpc_b64 s[66:67]\n.Lfar{n}:\n\ts_add_u32 s66, s66, ({lbl}-.Lfar{n})&4294967295"
                                  f"\n\ts_addc_u32 s67, s67, ({lbl}-.Lfar{n})>>32\n\ts_setpc_b64 s[66:67]"),
    "s_waitcnt_vm": lambda n: f"s_waitcnt vmcnt({n})",
    "s_waitcnt_lgkm": lambda: "s_waitcnt lgkmcnt(0)",
    "s_nop": lambda n: f"s_nop {n}",
    "s_setprio": lambda n: f"s_setprio {n}",
    # workgroups lo <= s2 < lo + width sleep iters x 127 x 64 cycles (s46/s47 scratch)
    "s_stagger": lambda lo, width, iters: (f"s_sub_u32 s46, s2, {lo}\n\ts_cmp_lt_u32 s46, {width}\n"
                                           f"\ts_cbranch_scc0 .Lstag_end\n\ts_mov_b32 s47, {iters}\n.Lstag:\n"
                                           f"\ts_sleep 127\n\ts_sub_u32 s47, s47, 1\n\ts_cmp_lg_u32 s47, 0\n"
                                           f"\ts_cbranch_scc1 .Lstag\n.Lstag_end:"),
    "s_load_args": lambda: "s_load_dwordx16 s[4:19], s[0:1], 0x0\n\ts_load_dwordx4 s[20:23], s[0:1], 0x40",
    "s_load_args_dec": lambda: "s_load_dwordx8 s[56:63], s[0:1], 0x50",
    "s_load_args_offs": lambda off: f"s_load_dwordx4 s[72:75], s[0:1], 0x{off:x}",
    "s_cmp_eq64_0_br": lambda s_, lbl: f"s_cmp_eq_u64 {SP(s_)}, 0\n\ts_cbranch_scc1 {lbl}",
    "load8": lambda d, a, off: f"global_load_dwordx2 {VP(d)}, {VP(a)}, off" + (f" offset:{off}" if off else ""),
    "v_add64_v": lambda d, a, b: f"v_lshl_add_u64 {VP(d)}, {VP(a)}, 0, {VP(b)}",
    "v_perm": lambda d, hi, lo, sel: f"v_perm_b32 {V(d)}, {V(hi)}, {V(lo)}, {V(sel)}",
    "v_perm_s": lambda d, hi, lo, s: f"v_perm_b32 {V(d)}, {V(hi)}, {V(lo)}, s{s}",
    "ds_read_b128": lambda d, a, off: f"ds_read_b128 {VQ(d)}, {V(a)}" + (f" offset:{off}" if off else ""),
    "ds_read_b32": lambda d, a, off: f"ds_read_b32 {V(d)}, {V(a)}" + (f" offset:{off}" if off else ""),
    "ds_write_b128": lambda a, d, off: f"ds_write_b128 {V(a)}, {VQ(d)}" + (f" offset:{off}" if off else ""),
    "s_waitcnt_lgkm_n": lambda n: f"s_waitcnt lgkmcnt({n})",
    "s_cmp_le_k_br": lambda s, kk, lbl: f"s_cmp_le_u32 s{s}, {kk}\n\ts_cbranch_scc1 {lbl}",
    "s_cmp_lg_k_br": lambda s, kk, lbl: f"s_cmp_lg_u32 s{s}, {kk}\n\ts_cbranch_scc1 {lbl}",
    "s_or64": lambda d, a, b: f"s_or_b64 {SP(d)}, {SP(a)}, {SP(b)}",
    "s_cmp_lg64_br": lambda s, lbl: f"s_cmp_lg_u64 {SP(s)}, 0\n\ts_cbranch_scc1 {lbl}",
    "s_endpgm": lambda: "s_endpgm",
    "s_barrier": lambda: "s_barrier",
    # synw (wave-uniform slot lookup): scalar map / base arithmetic, saddr loads
    "s_load_karg_x2": lambda d, off: f"s_load_dwordx2 {SP(d)}, s[0:1], 0x{off:x}",
    "s_load_x1": lambda d, a, off: f"s_load_dword s{d}, {SP(a)}, 0x{off:x}",
    "s_load_x2": lambda d, a, off: f"s_load_dwordx2 {SP(d)}, {SP(a)}, 0x{off:x}",
    "s_load_x4": lambda d, a, off: f"s_load_dwordx4 s[{d}:{d + 3}], {SP(a)}, 0x{off:x}",
    "s_addk": lambda d, a, k: f"s_add_u32 s{d}, s{a}, {k}",
    "s_add_cc": lambda d, a, b: f"s_add_u32 s{d}, s{a}, s{b}",
    "s_addc": lambda d, a, b: f"s_addc_u32 s{d}, s{a}, s{b}",
    "s_addck": lambda d, a, k: f"s_addc_u32 s{d}, s{a}, {k}",
    "s_mul_hi": lambda d, a, b: f"s_mul_hi_u32 s{d}, s{a}, s{b}",
    "s_max": lambda d, a, b: f"s_max_u32 s{d}, s{a}, s{b}",
    "s_lshr_s": lambda d, a, b: f"s_lshr_b32 s{d}, s{a}, s{b}",
    "s_bfe_k": lambda d, a, off, w: f"s_bfe_u32 s{d}, s{a}, 0x{off | (w << 16):x}",
    "s_cmp_eq_k": lambda a, k: f"s_cmp_eq_u32 s{a}, 0x{k:x}",
    "s_cselect64": lambda d, a, b: f"s_cselect_b64 {SP(d)}, {SP(a)}, {SP(b)}",
    "load16_saddr": lambda d, voff, sb, pol="": f"global_load_dwordx4 {VQ(d)}, {V(voff)}, {SP(sb)}"
                    + (f" {pol}" if pol else ""),
    # cmb (bit-sliced payload pass with wave-uniform runtime coefficients)
    "s_load_n": lambda d, base, n, soff, imm: (f"s_load_dword{'' if n == 1 else f'x{n}'} "
                                              + (f"s{d}" if n == 1 else f"s[{d}:{d + n - 1}]")
                                              + f", {SP(base)}, " + (f"s{soff}" if soff is not None else f"0x{imm:x}")
                                              + (f" offset:0x{imm:x}" if soff is not None and imm else "")),
    "s_sub": lambda d, a, b: f"s_sub_u32 s{d}, s{a}, s{b}",
    "s_cselect32": lambda d, a, b: f"s_cselect_b32 s{d}, s{a}, s{b}",
    "v_min_s": lambda d, s_, a: f"v_min_u32_e32 {V(d)}, s{s_}, {V(a)}",
    "s_idx_on": lambda s_: f"s_set_gpr_idx_on s{s_}, gpr_idx(SRC0)",
    "s_idx": lambda s_: f"s_set_gpr_idx_idx s{s_}",
    "s_idx_off": lambda: "s_set_gpr_idx_off",
    # jump-table products (KernelSpec.cmb_jump): the table's address, the call
    # and return, the block alignment and the destination-indexed XORs
    "s_getpc_rel": lambda d, lbl: (f"s_getpc_b64 s[{d}:{d + 1}]\n{lbl}_pc:\n\ts_add_u32 s{d}, s{d}, {lbl}-{lbl}_pc\n"
                                   f"\ts_addc_u32 s{d + 1}, s{d + 1}, 0"),
    "s_call": lambda ret, tgt: f"s_swappc_b64 s[{ret}:{ret + 1}], s[{tgt}:{tgt + 1}]",
    "s_ret": lambda ret: f"s_setpc_b64 s[{ret}:{ret + 1}]",
    "align7": lambda: ".p2align 7",
    "s_idx_on_d3": lambda s_: f"s_set_gpr_idx_on s{s_}, gpr_idx(SRC0,DST)",
    "s_idx_on_d2": lambda s_: f"s_set_gpr_idx_on s{s_}, gpr_idx(SRC1,DST)",
    "v_xor3_reld": lambda d, a, b: f"v_bitop3_b32 {V(d)}, {V(d)}, {V(a)}, {V(b)} bitop3:0x96",
    "v_xor_reld": lambda d, a: f"v_xor_b32_e32 {V(d)}, {V(a)}, {V(d)}",
    # d = v[base + M0] ^ b: src0 indexed while the gpr_idx mode is on
    "v_xor_rel": lambda d, base, b: f"v_xor_b32_e32 {V(d)}, {V(base)}, {V(b)}",
    "store16_saddr": lambda voff, d, sb, pol="": f"global_store_dwordx4 {V(voff)}, {VQ(d)}, {SP(sb)}"
                     + (f" {pol}" if pol else ""),
    "store_byte_saddr": lambda voff, d, sb, off: f"global_store_byte {V(voff)}, {V(d)}, {SP(sb)}"
                        + (f" offset:{off}" if off else ""),
    "store_byte": lambda a, d, off: f"global_store_byte {VP(a)}, {V(d)}, off" + (f" offset:{off}" if off else ""),
    # closed-form solve (cx): per-lane masked products on bit-planes
    "v_bfe_i": lambda d, a, off, w: f"v_bfe_i32 {V(d)}, {V(a)}, {off}, {w}",
    "v_and": lambda d, a, b: f"v_and_b32_e32 {V(d)}, {V(a)}, {V(b)}",
    # d = a ^ (b & c) (truth table index a*4 + b*2 + c)
    "v_xor_and": lambda d, a, b, c: f"v_bitop3_b32 {V(d)}, {V(a)}, {V(b)}, {V(c)} bitop3:0x78",
    "v_bcnt0": lambda d, a: f"v_bcnt_u32_b32 {V(d)}, {V(a)}, 0",
    "v_bcnt": lambda d, a, b: f"v_bcnt_u32_b32 {V(d)}, {V(a)}, {V(b)}",
    "v_cmp_ne0": lambda sd, a: f"v_cmp_ne_u32_e64 {SP(sd)}, 0, {V(a)}",
    # lab (lab_stamps): the real-time counter (100 MHz, chip-wide) into s[80 + 2p : 81 + 2p]
    "stamp": lambda p: f"s_memrealtime s[{STAMP_S0 + 2 * p}:{STAMP_S0 + 2 * p + 1}]",
    # lab (lab_stamps): the item's stores drained, stamp 7, then lane 0 writes
    # the 8 stamps and the wave's HW_ID / XCC_ID to stamps[item] (128 B each;
    # kernarg bytes 128..135) with vector stores; v14..v17 are dead there
    "stamp_flush": lambda: "\n\t".join(
        ["s_waitcnt vmcnt(0)", f"s_memrealtime s[{STAMP_S0 + 14}:{STAMP_S0 + 15}]",
         f"s_load_dwordx2 s[{STAMP_S0 + 16}:{STAMP_S0 + 17}], s[0:1], 0x{KERNARG_BYTES_DEC:x}",
         f"s_getreg_b32 s{STAMP_S0 + 18}, hwreg(HW_REG_HW_ID)",
         f"s_getreg_b32 s{STAMP_S0 + 19}, hwreg(HW_REG_XCC_ID)",
         "s_waitcnt lgkmcnt(0)", "s_lshl_b32 s66, s28, 7", "v_mov_b32_e32 v16, s66", "s_mov_b64 exec, 1"]
        + [f"v_mov_b32_e32 v14, s{STAMP_S0 + q}\n\tv_mov_b32_e32 v15, s{STAMP_S0 + q + 1}\n\t"
           f"global_store_dwordx2 v16, v[14:15], s[{STAMP_S0 + 16}:{STAMP_S0 + 17}] offset:{4 * q}"
           for q in (0, 2, 4, 6, 8, 10, 12, 14, 18)]
        + ["s_mov_b64 exec, -1"]),
    # lab: a cache-warming load (the destination is a dummy register)
    "load4": lambda d, a, off: f"global_load_dword {V(d)}, {VP(a)}, off" + (f" offset:{off}" if off else ""),
}


# --------------------------------------------------------------------------
# Kernel layout
# --------------------------------------------------------------------------
# Work unit: a wave handles one "item" of 128 consecutive 16-byte units of
# the flat (generation, unit) space; lane l owns units A = 128*item + l and
# B = A + 64, so every global_load_dwordx4 / store covers 1 KiB of
# consecutive units (two row segments at most).  A lane's two halves may
# belong to different generations: the encode coefficients are the same for
# all generations, and in syndrome mode each half gathers its own rows.
#
# kernarg (80 bytes, s4..s23):
#   s[4:5] src (syn: received rows)   s[6:7] dst (syn: syndrome rows)
#   s8  src generation stride (u32)   s9  dst generation stride (u32)
#   s10 src row stride                s11 dst row stride
#   s12 Lu = ceil(L/16) (payload units per row: lanes with u >= Lu load
#       nothing; a partial last unit is loaded whole -- the 16-B unit holding
#       byte L-1 never crosses a page -- and masked before the store)
#   s13 Lv >= Lu (lane units per row: the (generation, unit) lane space is
#       G x Lv; Lv = Lu rounded up to 8 puts every item boundary and row
#       start of a 128-B aligned layout on a 128-B line boundary)
#   s14 total units G*Lv   s15 magic (division by Lv)   s16 shift
#   s17 n_items   s18 total waves in the grid
#   s19 enc: units stored per row (Lu, or Lv: the zero tail [L, 16 Lv) of
#       each repair row is written too, so every stored line is whole);
#       syn: slot-map generation stride (syndromes of all Lv units are
#       stored: the syndrome rows live in the library's workspace)
#   s[20:21] slot map   s[22:23] zero row (syn)
#   s20..s23 enc: byte masks of the last unit's dwords (tail_masks(L))
# SGPRs: s[24:25] load mask B, s[26:27] load mask A, s28 item, s29 wave in
# group, s30 temp, s31 ABSENT constant, s[32:33] {src row stride, 0},
# s[34:35] {dst row stride, 0}, s[36:37] mad carry sink, s[38:39] and
# s[40:41] mask temps, s[48:49] store mask A, s[50:51] store mask B,
# s[52:53] mask temp.
KERNARG_BYTES = 96          # + s[72:75]: per-generation offset tables (see _gen_base)
V_LANE, V_F, V_GA, V_UA, V_GB, V_UB = 0, 1, 2, 3, 4, 5
V_SRCA, V_SRCB, V_DSTA, V_DSTB = 6, 8, 10, 12   # 64-bit pointers (even-aligned)
V_T = 14         # v14..v17 transpose temps
V_COMBO = 18     # 22 combo registers v18..v39
V_ZA, V_ZB, V_ADDR, V_SLOT = 40, 42, 44, 46      # syn only
SGPR_NEXT_FREE = 54
S_TMP, S_TMP2 = 38, 40
S_STA, S_STB, S_PAD = 48, 50, 52   # store masks of halves A / B, mask temp

# dec mode (fused decode: syndromes + in-register LU solve, see _generate_syn):
# extra kernarg dwords 20..27 at 0x50 -> s[56:63]:
#   s[56:57] LU records   s58 LU record stride   s59 L % 16 (lane-chunk decode; 0 otherwise)
#   s[60:61] split tables (256 x 32 B, gf256_tables.h perm_record)
#   s[62:63] {4096, 0} after the table copy (address constant)
# s64 jmax: 1 + the largest repair index any lane of the item has accepted.
KERNARG_BYTES_DEC = 128
SGPR_NEXT_FREE_DEC = 76      # s[66:67]: far-jump target, s68..s71: byte-pick selectors
# s[72:73] / s[74:75]: the source (syn / dec: received rows) and destination
# (dec: recovered rows) generation offset tables, or 0 (kernarg words at
# KERNARG_BYTES - 16 / KERNARG_BYTES_DEC - 16): generation g's base is then
# base + table[g] (64-bit byte offsets) instead of base + g * gen_stride --
# the heterogeneous batch API (qf_encode_batch_desc / qf_decode_batch_desc)
S_OFFS = 72
S_JMAX = 64
S_PICK = 68                  # v_perm selector placing byte b of a dword at bits 8..15
LDS_TAB_STRIDE = 256         # split-table record c at LDS byte c * 256 (address = byte << 8)
LDS_TAB_BYTES = 256 * LDS_TAB_STRIDE
LU_REC_BYTES = 272          # 16 columns x 16 B, then 16 rank bytes
KSPLIT_BLOCK_BYTES = 2048   # one accumulator block of a wave (8 dwords x 64 lanes) in LDS
# LU-phase VGPRs (regions free once the row loop is done; dec mode with
# r = 16: acc blocks v80..v207, slot maps v208..v247 are dead by then)
R_P = 14                    # 3 product temps (v14..v16)
R_SEL = 18                  # selectors s0[4], s1[4], s2[4] (v18..v29)
R_TB = (30, 36)             # table buffers T0lo T0hi T1lo T1hi T2 (v30..34, v36..40)
R_TA = (41, 42)             # their LDS addresses
R_FP = 44                   # LU record pointer (2)


def lu_layout(spec) -> tuple[list[int], tuple[int, int]]:
    """4-register slots of the LU phase in the ring and the slot maps (both
    dead after the row loop): the r columns of one half's record and the two
    halves' rank records.  Store addresses reuse the column slots."""
    slots = [spec.ring0 + 4 * q for q in range(2 * spec.nbuf)]
    slots += [spec.map_a + 4 * q for q in range(2 * spec.map_quads)]
    end = spec.map_b + 4 * spec.map_quads
    while len(slots) < spec.r + 2:     # small pd / k: extra registers past the maps
        slots.append(end)
        end += 4
    return slots[2: 2 + spec.r], (slots[0], slots[1])
# synw mode (wave-uniform slot lookup, _generate_synw): kernarg words 24..25
# (byte 0x60) = per-generation bound (1 + the largest accepted repair index,
# k_decode_prepare_cauchy) or 0.  An item's units lie in generations g0 and
# g1 = min(g0 + 1, G - 1); per row, the scalar unit reads both generations'
# slot bytes and forms each one's row address (zero row if absent), and the
# halves load with that address as saddr under the lanes of each generation.
KERNARG_BYTES_SYNW = 104
SW_A0, SW_A1, SW_B0, SW_B1 = 54, 56, 58, 60   # load lanes: half A / B x generation g0 / g1
SW_R0, SW_R1 = 62, 64                         # received-row bases of g0 / g1
SW_M0, SW_M1 = 68, 70                         # slot-map pointers of g0 / g1
SW_BOUND = 76                                 # s[76:77] bound table (kernarg)
SW_G0, SW_G1, SW_GLAST = 78, 79, 80           # g0, g1, G - 1
SW_Q0, SW_Q1 = 84, 88                         # the current map quad of g0 / g1 (4 SGPRs each)
SW_BASE0, SW_BASE1 = 92, 94                   # this row's address in g0 / g1
SW_T0, SW_T1 = 96, 97                         # slot bytes / temps
SW_NEXT_FREE = 98
STAMP_S0 = 82    # lab_stamps: s82..s97 stamps, s[98:99] buffer, s100 / s101 HW_ID / XCC_ID (above S_ROWLDS)
S_TMASK = 42     # s42..s44: the transpose masks 0x0F0F0F0F, 0x33333333, 0x55555555
S_ABSENT = 31    # holds ABSENT (VOP3 takes no literal)
ABSENT = 0xFF    # slot-map value of a row that was not accepted


@dataclasses.dataclass
class KernelSpec:
    k: int
    r: int
    pd: int = 3
    mode: str = "enc"   # "enc": repairs of the Cauchy code; "syn": decode syndromes;
    # "synw": decode syndromes with the slot map read per row by the scalar unit
    # (an item spans at most two generations: padded row units >= 128)
    xor3: bool = True   # acc ^= L ^ H as one v_bitop3_b32 (3-input XOR, full rate)
    # cache policy of the streamed rows: read once / written once, so
    # non-temporal (tools/bs_lab.py: -9 % at C2 vs the default policy)
    ld_policy: str = "nt"
    st_policy: str = "nt"
    # transpose swaps as shift + bit-select (4 ops per pair) instead of the
    # classic xor/and/xor delta swap (6 ops per pair)
    bfi_transpose: bool = True
    # workgroup w processes items of a contiguous range per XCD (blocks go to
    # XCD w % 8), so lines shared by neighbouring items meet in one L2
    xcd_remap: bool = True
    # dec mode: accumulator blocks j >= guard_min are skipped when no lane of
    # the item has accepted repair j (j >= jmax)
    guard_min: int = 4
    # dec mode: solve in registers (False: store the syndromes unsolved; lab only)
    lu: bool = True
    # dec mode: wave priority (s_setprio) of the row loop / the LU phase
    prio: tuple = (0, 0)
    # (lo, width, iters): workgroups lo..lo+width-1 sleep about iters x 8 k cycles
    # before their first item, so co-resident waves run their memory (row loop) and
    # compute (LU) phases out of step instead of in lock-step
    stagger: tuple = ()
    # lab only: drop the payload row loads (keeps maps, records, compute)
    lab_norows: bool = False
    # lab only (chunked dec): absent rows read zero row (g & 63) of a region of
    # 64 zero rows 2,048 B apart instead of one shared zero row (spreads the
    # ~20 % of row loads that hit it over 64 x 10 lines)
    lab_zspread: bool = False
    # lab only (chunked dec): skip the row loop (the LU phase alone, on whatever
    # the accumulator registers hold) -- timing of the LU in isolation
    lab_lu_only: bool = False
    # lab only (chunked fft dec): row n of the loop reads slot n % 64 of the
    # generation (no slot map: the generation's rows in address order; the
    # results are wrong, timing of the access pattern only)
    lab_slot_order: bool = False
    # lab only (chunked fft dec): absent rows are not loaded at all (their
    # lanes masked off) instead of reading the shared zero row
    lab_skip_absent: bool = False
    # lab only (chunked dec, Q = 2^m lane-chunks, recovered rows >= 32 Q bytes
    # apart): every lane of a generation stores its B half, the lanes past the
    # last unit included (the zero tail of pool-block rows: whole 128-B lines)
    lab_full_b_store: bool = False
    # lab only (chunked dec): "fwd" / "bwd" -- only the forward (L, diagonal)
    # or only the backward (U') products of the LU run (results wrong; the
    # marginal time of ~half the per-lane products)
    lab_lu_part: str = ""
    # lab only (fft row loop): the first n chunks' transposes, butterflies and
    # folds dropped (their rows still load): the marginal time of row-loop VALU
    lab_skip_chunks: int = 0
    # lab only (chunked dec): the split tables at a 32-B record stride (8 KB,
    # records start on 8 different LDS banks) instead of 256 B (64 KB, every
    # record on the same bank)
    lab_tab32: bool = False
    # lab only (cmb): "idx_once" -- one index row per input row, reused by every
    # output (no per-product scalar load); "noload" -- no input-row loads
    lab_cmb: tuple = ()
    # cmb: the gpr_idx mode on for a row's whole product run (not per product)
    # and the early exit tested every 4 outputs (products past a generation's
    # outputs go to accumulators that are never stored)
    cmb_lean: bool = False
    # cmb (R <= 16): input rows prefetched two ahead (a third row buffer at
    # v192..v199: 200 VGPRs, still two waves per SIMD)
    cmb_pf2: bool = False
    # cmb (R <= 16): the product of a row by output j's runtime coefficient c
    # as a call into c's code block (256 blocks of 128 B after the kernel's
    # end, built from cmb_index_table), accumulator set j chosen by the gpr_idx
    # index 8 j on the destination: 3 = 8 VOP3 xor3 (acc ^= LO[a] ^ HI[b]) per
    # block; 2 = 16 VOP2 xors; 0 = M0-indexed sources (an s_set_gpr_idx_idx per
    # XOR). 6 SALU per product instead of 16 + the index-row load
    cmb_jump: int = 0
    # enc: the library's sliding-window variant of a shape ('g', chosen when a
    # batch's generations overlap): "_sl" appended to the name
    sliding: bool = False
    # VALU list scheduling (bs_sched.schedule): runs of plain VALU ops between
    # non-VALU ops reordered so a producer sits >= sched ops before its
    # consumers where the run allows it (0: program order)
    sched: int = 0
    # chunked dec, small batches: the four waves of a workgroup share ONE item,
    # each running every ksplit-th row of it; waves 1..3 hand their partial
    # syndromes to wave 0 through LDS, which solves and stores (kernel
    # qf_cauchy_decs_*: a generation's rows no longer run through one wave)
    ksplit: int = 1
    # chunked dec: LU products of 2-3 dwords interleaved (their v_perm results in
    # separate temps) and selectors issued stage by stage, so that dependent
    # VALU ops sit several instructions apart
    lu_ilp: bool = False
    # chunked fft dec: split-table reads in flight ahead of the LU products
    # (1: the next coefficient's; 2: the next two, a third table buffer in
    # the registers the record pointer and the second address held)
    lu_ahead: int = 1
    # lab only (chunked dec, strided rows): (n_slots, 16 Q) -- during the
    # backward LU phase, touch every row the NEXT item will read (one dword
    # load per half and row into a dummy register), so that its row loop finds
    # them in L2 / the Infinity Cache while HBM would otherwise idle
    lab_prefetch: tuple = ()
    # chunked fft dec: the closed-form Cauchy solve (round 6): x_E = alpha *
    # (C^T (beta * s))|_E, C^T through the additive-FFT plan run backwards
    # with every op transposed, alpha / beta per-lane masked products on the
    # bit-planes (no LU, no split tables); cx records (cx_record) instead of
    # LU records
    cx: bool = False
    # lab only (chunked fft dec): per-item phase timestamps (s_memrealtime)
    # written to a buffer named by kernarg bytes 128..135 (tools/dec_lab.py
    # --stamps): entry, item start, map read, source rows done, repairs done,
    # forward LU done, backward LU + stores issued, stores drained
    lab_stamps: bool = False
    # enc mode, one pass of a code with more repairs than a kernel holds:
    # repairs j0 .. j0 + r - 1 of the Cauchy matrix of (k, r_total)
    r_total: int = 0
    j0: int = 0
    # dec mode, lane-chunk layout: lane l of item w owns units q and q + Q of
    # ONE generation (f = 64 w + l, g = f / Q, q = f % Q, Q = ceil(Lu / 2)),
    # so each lane has one slot map, one LU record and one table read per
    # coefficient for both 16-byte halves (_generate_dec_chunked)
    chunked: bool = False
    # lab only (chunked): one generation per wave (item = generation, lanes
    # q < Q active), so row presence is wave-uniform and the row loop skips
    # the erased sources (tools/dec_lab.py)
    wave_gen: bool = False
    # transpose masks in VGPRs (all-VGPR v_bitop3 issues at full rate, with an
    # SGPR operand at half: tools/ubench_idx.py, profiles/r02_ubench_idx.json)
    vgpr_masks: bool = True
    # additive-FFT row loop (k a power of two, lch_fft.py): sources stream in
    # chunks of `fft` rows, each chunk is inverse-transformed in registers and
    # folded into R coset accumulators, a final transform gives the repairs
    # (enc) / syndromes (chunked dec).  0: one coefficient block per repair
    fft: int = 0
    # fft: the end-of-chunk work (last butterflies + folds into the
    # accumulators) is spread over the next fft_defer rows, so loads keep
    # being issued through it (needs fft_defer more ring slots)
    fft_defer: int = 0
    # chunked dec with fft: rows land in LDS (global_load_lds_dwordx4, no VGPR
    # destination) in lds_rows slots per wave, so lds_rows - 1 rows are in
    # flight whatever the register budget; the split tables then sit at a
    # 32-B stride (8 KB per workgroup instead of 64 KB)
    lds_rows: int = 0
    # fft: (basis, beta_out) of the plan; () = lch_fft.BEST (or canonical)
    fft_basis: tuple = ()
    # chunked dec: store each recovered row as soon as back-substitution has
    # finished it (x_u after backward column u), not all after the solve
    early_stores: bool = False
    # fft: plane pairs shared by >= 3 output rows of a constant multiply are
    # XORed once into the transpose scratch registers
    fft_cse: bool = True
    # fft passes of codes the plain plan does not cover (lch_fft.hybrid_plan):
    # repair points per coset, i.e. accumulator blocks (16, or 8: half the
    # accumulator VGPRs, twice the passes)
    fft_coset: int = 16
    # enc: this pass is one wave of a MergedSpec dispatch (item = workgroup,
    # the workgroup's waves run the code's passes on the same item)
    merged: bool = False
    # this pass is one block range of a pass-major MergedSpec (concat): the
    # usual prologue, with the end of the common head marked
    head_mark: bool = False
    # cmb: every pass of the payload in one pass-major launch (the grid holds
    # the passes' workgroup ranges; kernarg word 32 = the coefficient records'
    # pass stride)
    pass_major: bool = False
    # cmb pass-major, item-major interleave: the P passes of one persistent
    # slot are neighbouring workgroups on one XCD (workgroup w: XCD w % 8, pass
    # (w >> 3) mod P, slot 8 ((w >> 3) div P) + w % 8), so they walk the same
    # items together and the later passes' syndrome reads hit that XCD's L2;
    # kernarg word 33 = (ceil(2^16 / P) << 3) | P, the grid a multiple of 8 P
    pm_xcd: bool = False
    # enc fft, one pass of a MergedSpec built with xchg: (waves, this wave).
    # The pass-independent row work (loads, transposes, the chunks' inverse
    # butterflies) is split over the workgroup's waves by chunk and handed
    # over in LDS; each wave folds every chunk into its own pass's
    # accumulators (_generate_enc_xchg)
    xchg: tuple = ()
    # xchg: rows of a wave's next group whose loads are issued before it
    # transforms its current group (the rest after, as its registers free up):
    # the row slots grow from ch + 2 to ch + early, so a load has a produce and
    # a fold phase to land in instead of a fold phase
    xchg_early: int = 0

    @property
    def ahead(self) -> int:
        """Rows loaded ahead of the one being processed."""
        return self.lds_rows - 1 if self.lds_rows else self.pd

    @property
    def tab_stride(self) -> int:
        return 32 if self.lds_rows or self.lab_tab32 else LDS_TAB_STRIDE

    @property
    def fplan(self):
        if not self.fft:
            return None
        if self.fft_basis:
            from . import lch_fft
            return lch_fft.plan(self.k, self.r, self.fft, basis=self.fft_basis[0], beta_out=self.fft_basis[1])
        if self.k & (self.k - 1) or self.rt != self.r or self.j0:
            # a pass of a code the plain plan does not cover (lch_fft.hybrid_plan)
            return _hybrid_plan(self.k, self.rt, self.j0, self.r, self.fft, self.fft_coset)
        return _fft_plan(self.k, self.r, self.fft)

    @property
    def nacc(self) -> int:
        """Accumulator blocks of 8 planes: the r repairs, or the plan's R."""
        return self.fplan.R if self.fft else self.r

    @property
    def vmask(self) -> Optional[tuple]:
        """VGPRs holding the transpose masks 0x0F0F0F0F, 0x33333333, 0x55555555
        (None: SGPRs s42..s44).  The lane-chunk decode uses registers its
        layout leaves free (V_DSTB pair, V_ZB); the others append three."""
        if not self.vgpr_masks or self.mode == "cmb":
            return None
        if self.mode == "dec" and self.chunked:
            return (V_DSTB, V_DSTB + 1, V_ZB)
        n = self._base_free_vgpr()
        if n + 3 > 256:   # no room: the masks stay in SGPRs
            return None
        return (n, n + 1, n + 2)

    @property
    def rt(self) -> int:
        return self.r_total or self.r

    @property
    def name(self) -> str:
        if self.mode == "cmb":
            return (f"qf_combine_bs_r{self.r}" + ("_pmx" if self.pm_xcd else "_pm" if self.pass_major else "")
                    + (f"_j{self.cmb_jump}" if self.cmb_jump else ""))
        tag = {"enc": "bss" if self.ksplit > 1 else "bs", "syn": "syn", "dec": "dec", "synw": "synw"}[self.mode]
        if self.chunked:
            tag = "decs" if self.ksplit > 1 else ("decx" if self.cx else "decc")
        if self.fft:
            tag += f"f{self.fft}" + (f"l{self.lds_rows}" if self.lds_rows else "")
        sl = "_sl" if self.sliding else ""
        if self.rt != self.r or self.j0:
            return f"qf_cauchy_{tag}_k{self.k}_r{self.rt}_j{self.j0}{sl}"
        return f"qf_cauchy_{tag}_k{self.k}_r{self.r}{sl}"

    @property
    def nbuf(self) -> int:
        # fft: a chunk's rows stay in the ring until it is folded in, while the
        # next chunk's first pd rows land
        if self.fft and self.lds_rows:
            return self.fft          # only the chunk itself lives in registers
        if self.xchg:
            # the chunk being produced + two rows read back from LDS (+ the
            # next group's early rows beyond those two)
            return self.fft + max(2, self.xchg_early)
        return self.pd + (self.fft + self.fft_defer if self.fft else 1)

    @property
    def ring0(self) -> int:
        if self.fft:     # no plane-combination registers (v18..v39)
            return FFT_RING0_DEC if self.mode == "dec" else FFT_RING0_ENC
        return 40 if self.mode == "enc" else 48

    @property
    def acc0(self) -> int:
        return self.ring0 + 8 * self.nbuf

    @property
    def map_quads(self) -> int:
        """Slot-map quads held in VGPRs per half (synw reads the map with scalar loads)."""
        return (self.k + self.r + 15) // 16 if self.mode in ("syn", "dec") else 0

    @property
    def n_maps(self) -> int:
        return 1 if self.chunked else 2

    @property
    def map_a(self) -> int:
        if self.fft and self.mode == "dec":
            return FFT_MAP_DEC      # the plane-combination registers are free
        return self.acc0 + 8 * self.nacc

    @property
    def map_b(self) -> int:
        return self.map_a + (0 if self.chunked else 4 * self.map_quads)

    @property
    def map_stride(self) -> int:
        """Bytes per generation in the slot map (k source + r repair slots)."""
        if self.mode == "synw":
            return 16 * ((self.k + self.rt + 15) // 16)
        return 16 * self.map_quads

    def _base_free_vgpr(self) -> int:
        n = self.map_b + 4 * self.map_quads
        if self.fft:
            n = max(n, self.acc0 + 8 * self.nacc)
        if self.mode == "dec" and self.chunked and self.cx:
            n = max(n, cx_alpha0(self) + 4 * ((self.k + 15) // 16))
        elif self.mode == "dec" and self.chunked:
            n = max(n, lu_layout_chunked(self)["end"])
        elif self.mode == "dec":
            n = max(n, max(lu_layout(self)[0]) + 4)
        return n

    @property
    def next_free_vgpr(self) -> int:
        if self.mode == "cmb":
            return _cmb_regs(self.r)["end"] + (8 if self.cmb_pf2 else 0)
        n = self._base_free_vgpr()
        if self.vmask is not None and not (self.mode == "dec" and self.chunked):
            n += 3
        if (self.lds_rows and self.mode == "enc") or self.xchg:
            n += 1          # the ds_read address of the row slots
        n = (n + 7) // 8 * 8
        if n > 256:
            raise ValueError(f"{self.name}: {n} VGPRs > 256 (lower pd)")
        return n

    @property
    def next_free_sgpr(self) -> int:
        if self.mode == "cmb":
            return CMB_NEXT_FREE_SGPR
        if self.mode == "synw":
            return SW_NEXT_FREE
        if self.mode == "dec" and self.lab_stamps:
            return STAMP_S0 + 20
        if self.mode == "dec":
            # chunked: s[76:77] = {16 Q, 0}, s[78:79] the partial-last-unit lane
            return SGPR_NEXT_FREE_DEC + (4 if self.chunked else 0) + (2 if self.lds_rows else 0)
        # s[66:67]: far-jump target, s[72:75]: offset tables (+ s76: LDS row base)
        return S_OFFS + 4 + (2 if self.lds_rows else 0)

    @property
    def far(self) -> bool:
        """Item loop branches as 64-bit pc-relative jumps: the straight-line
        body exceeds the +-128 KiB of s_branch (dec always; enc / syn for large k*r)."""
        return self.mode == "dec" or bool(self.fft) or self.k * (70 + 8 * self.r) > 14000

    @property
    def kernarg_bytes(self) -> int:
        if self.mode == "cmb":
            return KERNARG_BYTES_CMB + (8 if self.pass_major or self.r > 16 else 0)
        if self.mode == "synw":
            return KERNARG_BYTES_SYNW
        if self.mode == "dec" and self.lab_stamps:
            return KERNARG_BYTES_DEC + 16
        return KERNARG_BYTES_DEC if self.mode == "dec" else KERNARG_BYTES

    @property
    def offs_kernarg(self) -> int:
        """Byte offset of the generation offset tables in the kernarg block
        (lab_stamps: the stamp buffer pointer follows them)."""
        if self.mode == "dec" and self.lab_stamps:
            return KERNARG_BYTES_DEC - 16
        return KERNARG_BYTES - 16 if self.mode == "synw" else self.kernarg_bytes - 16

    @property
    def lds_bytes(self) -> int:
        if self.mode == "dec" and self.ksplit > 1:
            return LDS_TAB_BYTES + (self.ksplit - 1) * self.r * KSPLIT_BLOCK_BYTES
        if self.mode == "enc" and self.ksplit > 1:
            return (self.ksplit - 1) * self.r * KSPLIT_BLOCK_BYTES
        if self.mode == "dec" and self.cx and not self.lds_rows:
            return 0
        if self.mode == "dec" and self.lds_rows:
            return (0 if self.cx else 256 * self.tab_stride) + 4 * self.lds_rows * LDS_ROW_BYTES
        if self.mode == "dec" and self.lab_tab32 and self.ksplit == 1:
            return 256 * self.tab_stride
        if self.mode == "enc" and self.lds_rows:
            return 4 * self.lds_rows * LDS_ROW_BYTES
        if self.xchg:
            return self.xchg[0] * self.fft * LDS_ROW_BYTES
        return LDS_TAB_BYTES if self.mode == "dec" else 0


_TRANSPOSE = [(4, 0x0F0F0F0F, [(0, 4), (1, 5), (2, 6), (3, 7)]),
              (2, 0x33333333, [(0, 2), (1, 3), (4, 6), (5, 7)]),
              (1, 0x55555555, [(0, 1), (2, 3), (4, 5), (6, 7)])]

# combo register for nonzero 4-bit masks (low group L, high group H)
_COMBO_BUILD = {  # mask: (a, b) meaning combo = a ^ b, where a/b are masks
    3: (1, 2), 5: (1, 4), 6: (2, 4), 7: (3, 4), 9: (1, 8), 10: (2, 8), 11: (3, 8),
    12: (4, 8), 13: (12, 1), 14: (12, 2), 15: (7, 8),
}


def _transpose_ops(base: int, bfi: bool = False, vmask: Optional[tuple] = None) -> list[Op]:
    """32 bytes in 8 dwords <-> 8 bit-planes (3 delta-swap stages; an
    involution, so the same network maps planes back to bytes).

    bfi: each swap of (a, b) with shift s and mask M is
      a' = (M & a) | (~M & (b << s)),  b' = (M & (a >> s)) | (~M & b)
    i.e. two shifts and two v_bitop3 bit-selects with M in an SGPR, or in
    the VGPR vmask[stage] when the kernel keeps the masks in VGPRs."""

    def sel(d, stage, a, b):
        if vmask is not None:
            return Op("v_bitsel_v", (d, vmask[stage], a, b))
        return Op("v_bitsel_s", (d, S_TMASK + stage, a, b))
    ops = []
    if bfi == "s64":
        # stages 1 and 2 shift register pairs with one 64-bit shift: the bits a
        # v_lshlrev_b64 carries into the high dword land where the bit-select
        # takes the other operand (and likewise for the right shift into the
        # low dword), so they never reach the result
        for stage, (sh, mask, pairs) in enumerate(_TRANSPOSE):
            sm = S_TMASK + stage
            if stage == 2:
                for q, (a, b) in enumerate(pairs):
                    t, u = V_T + 2 * (q & 1), V_T + 2 * (q & 1) + 1
                    ops.append(Op("v_lshl", (t, sh, base + b)))
                    ops.append(Op("v_lshr", (u, sh, base + a)))
                    ops.append(sel(base + a, stage, base + a, t))
                    ops.append(sel(base + b, stage, u, base + b))
                continue
            for q in range(0, 4, 2):
                (a0, b0), (a1, b1) = pairs[q], pairs[q + 1]
                assert a1 == a0 + 1 and b1 == b0 + 1 and (base + a0) % 2 == 0 and (base + b0) % 2 == 0
                ops.append(Op("v_lshl64", (V_T, sh, base + b0)))        # t pair = (b0, b1) << sh
                ops.append(Op("v_lshr64", (V_T + 2, sh, base + a0)))    # u pair = (a0, a1) >> sh
                for x, (a, b) in enumerate(((a0, b0), (a1, b1))):
                    ops.append(sel(base + a, stage, base + a, V_T + x))
                    ops.append(sel(base + b, stage, V_T + 2 + x, base + b))
        return ops
    if bfi:
        for stage, (sh, mask, pairs) in enumerate(_TRANSPOSE):
            sm = S_TMASK + stage
            for q, (a, b) in enumerate(pairs):
                t, u = V_T + 2 * (q & 1), V_T + 2 * (q & 1) + 1
                ops.append(Op("v_lshl", (t, sh, base + b)))
                ops.append(Op("v_lshr", (u, sh, base + a)))
                ops.append(sel(base + a, stage, base + a, t))
                ops.append(sel(base + b, stage, u, base + b))
        return ops
    for sh, mask, pairs in _TRANSPOSE:
        t = [V_T + q for q in range(4)]
        ops += [Op("v_lshr", (t[q], sh, base + a)) for q, (a, b) in enumerate(pairs)]
        ops += [Op("v_xor", (t[q], t[q], base + b)) for q, (a, b) in enumerate(pairs)]
        ops += [Op("v_andk", (t[q], mask, t[q])) for q, (a, b) in enumerate(pairs)]
        ops += [Op("v_xor", (base + b, base + b, t[q])) for q, (a, b) in enumerate(pairs)]
        ops += [Op("v_lshl", (t[q], sh, t[q])) for q, (a, b) in enumerate(pairs)]
        ops += [Op("v_xor", (base + a, base + a, t[q])) for q, (a, b) in enumerate(pairs)]
    return ops


def _combo_regs(base: int) -> tuple[dict, dict]:
    """Register of each nonzero 4-bit combination: singles are the planes."""
    lo = {1: base + 0, 2: base + 1, 4: base + 2, 8: base + 3}
    hi = {1: base + 4, 2: base + 5, 4: base + 6, 8: base + 7}
    nxt = V_COMBO
    for m in sorted(_COMBO_BUILD):
        lo[m] = nxt
        nxt += 1
    for m in sorted(_COMBO_BUILD):
        hi[m] = nxt
        nxt += 1
    return lo, hi


def _combo_ops(lo: dict, hi: dict, needed_lo: set, needed_hi: set) -> list[Op]:
    ops = []
    for tab, need in ((lo, needed_lo), (hi, needed_hi)):
        # close the needed set under the build dependencies
        want = set(need)
        changed = True
        while changed:
            changed = False
            for m in list(want):
                if m in _COMBO_BUILD:
                    for d in _COMBO_BUILD[m]:
                        if d not in want:
                            want.add(d)
                            changed = True
        for m in sorted(_COMBO_BUILD):
            if m in want:
                a, b = _COMBO_BUILD[m]
                ops.append(Op("v_xor", (tab[m], tab[a], tab[b])))
    return ops


def _coeff_block(ops: list[Op], rows_j: list[int], acc: int, lo: dict, hi: dict, init: bool,
                 xor3: bool = False):
    """acc[b] (^)= M_c[b] * planes for one coefficient (rows_j = M_c rows)."""
    first_pass, second = [], []
    for b in range(8):
        a = acc + b
        m_lo, m_hi = rows_j[b] & 15, rows_j[b] >> 4
        if init:
            if m_lo and m_hi:
                first_pass.append(Op("v_xor", (a, lo[m_lo], hi[m_hi])))
            elif m_lo:
                first_pass.append(Op("v_mov", (a, lo[m_lo])))
            elif m_hi:
                first_pass.append(Op("v_mov", (a, hi[m_hi])))
            else:
                first_pass.append(Op("v_movk", (a, 0)))
        elif xor3 and m_lo and m_hi:
            first_pass.append(Op("v_xor3", (a, a, lo[m_lo], hi[m_hi])))
        else:
            if m_lo:
                first_pass.append(Op("v_xor", (a, a, lo[m_lo])))
            if m_hi:
                (second if m_lo else first_pass).append(Op("v_xor", (a, a, hi[m_hi])))
    ops.extend(first_pass + second)


def _source_row(ops: list[Op], C, i: int, r: int, base: int, acc0: int, init: bool, xor3: bool = False,
                bfi: bool = False, guard: Optional[tuple[int, str]] = None, vmask: Optional[tuple] = None):
    """Transpose one source row (ring buffer at `base`) and accumulate it into
    all r repair accumulators with the Cauchy coefficients of column i.
    guard = (j0, label): blocks j >= j0 are skipped (jump to label) once
    j >= jmax (dec mode)."""
    ops.extend(_transpose_ops(base, bfi, vmask))
    lo, hi = _combo_regs(base)
    rows = [mul_matrix_rows(C[j][i]) for j in range(r)]
    need_lo = {rb & 15 for rr in rows for rb in rr} - {0}
    need_hi = {rb >> 4 for rr in rows for rb in rr} - {0}
    ops.extend(_combo_ops(lo, hi, need_lo, need_hi))
    for j in range(r):
        if guard is not None and j >= guard[0]:
            ops.append(Op("s_cmp_le_k_br", (S_JMAX, j, guard[1])))
        _coeff_block(ops, rows[j], acc0 + 8 * j, lo, hi, init, xor3)
    if guard is not None and guard[0] < r:
        ops.append(Op("label", (guard[1],)))


# --------------------------------------------------------------------------
# Additive-FFT row loop (spec.fft, lch_fft.py)
# --------------------------------------------------------------------------
FFT_RING0_ENC = 18     # the ring starts where the plane combinations lived
FFT_RING0_DEC = 48     # chunked dec keeps its low registers (V_ZA .. v47)
FFT_MAP_DEC = 18       # chunked dec: slot map quads v18..v37 (dead in the LU phase)
FFT_MAP_DEC_QUADS = 5  # ... k + r <= 80 slots; larger maps run a window of 5 quads there
LDS_ROW_BYTES = 2048   # lds_rows: one row of a wave (64 lanes x 2 units x 16 B) per LDS slot
S_ROWLDS = 80          # lds_rows: the wave's first LDS row slot (byte address)
S_ROWLDS_ENC = 76      # the same in the encode kernels
V_LDSA = 47            # lds_rows: S_ROWLDS + 16 lane (ds_read address of the A half)


def _fft_plan(k: int, r: int, ch: int):
    from . import lch_fft
    return lch_fft.best_plan(k, r, ch)


@functools.lru_cache(maxsize=None)
def _hybrid_plan(k: int, rt: int, j0: int, r: int, ch: int, R: int = 16):
    from . import lch_fft
    return lch_fft.hybrid_plan(k, rt, j0, r, ch, R)


def _macc_cost(c: int, n_tmp: int = 0) -> int:
    if c == 0:
        return 0
    if c == 1:
        return 8
    temps, terms = _cse_pairs(mul_matrix_rows(c), n_tmp)
    return len(temps) + sum((len(t) + 1) // 2 for t in terms)


def _cse_pairs(rows: list[int], n_tmp: int) -> tuple[list, list]:
    """Greedy common-subexpression pass over the rows of M_c: a pair of input
    planes shared by >= 3 output rows becomes one temp (1 XOR, and one term
    less in each of those rows: ~n/2 ops saved).  Returns the temps [(a, b)]
    (operands: plane index 0..7 or 8 + temp) and each row's term list."""
    terms = [[a for a in range(8) if w >> a & 1] for w in rows]
    temps = []
    while len(temps) < n_tmp:
        cnt = {}
        for t in terms:
            for i in range(len(t)):
                for j in range(i + 1, len(t)):
                    cnt[(t[i], t[j])] = cnt.get((t[i], t[j]), 0) + 1
        if not cnt:
            break
        (a, b), n = max(sorted(cnt.items()), key=lambda kv: kv[1])
        if n < 3:
            break
        x = 8 + len(temps)
        temps.append((a, b))
        for t in terms:
            if a in t and b in t:
                t.remove(a)
                t.remove(b)
                t.append(x)
    return temps, terms


def _macc(E, dst: int, src: int, c: int, init: bool, tmp: tuple = ()):
    """dst (8 planes) ^= c * src, or dst = c * src when init (c a compile-time
    GF(256) constant: output plane b is the XOR of the input planes of row b
    of M_c, two per v_bitop3).  tmp: scratch VGPRs for shared plane pairs."""
    rows = mul_matrix_rows(c)
    temps, rterms = _cse_pairs(rows, len(tmp)) if tmp and c not in (0, 1) else ([], None)

    def reg(a):
        return src + a if a < 8 else tmp[a - 8]
    for q, (a, b) in enumerate(temps):
        E(Op("v_xor", (tmp[q], reg(a), reg(b))))
    for b in range(8):
        d = dst + b
        terms = [reg(a) for a in rterms[b]] if rterms is not None else \
            [src + a for a in range(8) if rows[b] >> a & 1]
        if init:
            if not terms:
                E(Op("v_movk", (d, 0)))
                continue
            if len(terms) == 1:
                E(Op("v_mov", (d, terms[0])))
                continue
            if len(terms) == 2:
                E(Op("v_xor", (d, terms[0], terms[1])))
                terms = []
            else:
                E(Op("v_xor3", (d, terms[0], terms[1], terms[2])))
                terms = terms[3:]
        while len(terms) >= 2:
            E(Op("v_xor3", (d, d, terms[0], terms[1])))
            terms = terms[2:]
        if terms:
            E(Op("v_xor", (d, d, terms[0])))


def _fft_stream(E, ops: list, spec: KernelSpec, load_row, wait_row, acc_block, n_rows: int = 0):
    """The additive-FFT row loop: plan row n (source plan.order[n]) lands in
    ring slot n % nbuf, is transposed to planes, the chunk's inverse
    butterflies run as soon as both operands are complete, the chunk is folded
    into the accumulators after its last row, and the final forward
    butterflies run after the last chunk.  load_row(n, base) issues the loads
    of plan row n into the ring slot at `base`; wait_row(n) waits for them;
    acc_block(t) is the first register of accumulator t.  n_rows > k: rows
    k .. n_rows - 1 (processed by the caller) are prefetched as well."""
    P = spec.fplan
    k, ch, pd, nbuf = spec.k, P.ch, spec.ahead, spec.nbuf
    n_rows = max(n_rows, k)
    ring0 = spec.ring0

    def slot(n):
        return ring0 + 8 * (n % nbuf)

    # butterflies of each chunk by the chunk row after which they are ready
    ready = []
    for bf in P.chunk_bfly:
        by_m = {}
        for i, j, s in bf:
            q = (j - i).bit_length() - 1
            m = (i - i % (2 << q)) + (2 << q) - 1
            by_m.setdefault(m, []).append((i, j, s))
        ready.append(by_m)
    inited = set()
    defer = spec.fft_defer
    assert defer < ch
    last_q = ch.bit_length() - 2          # the chunk's last (top) inverse layer

    tmp = tuple(range(V_T, V_T + 4)) if spec.fft_cse else ()

    def butterfly(base, i, j, s):
        yi, yj = slot(base + i), slot(base + j)
        for b in range(8):
            E(Op("v_xor", (yj + b, yj + b, yi + b)))
        if s:
            _macc(E, yi, yj, s, init=False, tmp=tmp)

    def fold(hc, mm):
        for t, c in P.acc[(hc, mm)]:
            _macc(E, acc_block(t), slot(hc * ch + mm), c, init=t not in inited, tmp=tmp)
            inited.add(t)

    groups = []      # deferred end-of-chunk work, one group per following row
    for n in range(min(pd, n_rows)):
        load_row(n, slot(n))
    kA = getattr(P, "kA", 0) or k        # plan rows through the FFT; rows kA .. k - 1 enter directly
    direct = getattr(P, "direct", {})

    def fold_direct(n):
        for t, c in direct[n]:
            _macc(E, acc_block(t), slot(n), c, init=t not in inited, tmp=tmp)
            inited.add(t)

    for n in range(k):
        if n + pd < n_rows:
            load_row(n + pd, slot(n + pd))
        wait_row(n)
        if n < spec.lab_skip_chunks * ch:
            continue
        ops.extend(_transpose_ops(slot(n), spec.bfi_transpose, spec.vmask))
        if n >= kA:
            work = [(0, lambda n=n: fold_direct(n))]
            if groups:
                work = [(0, e) for e in groups.pop(0)] + work
            for _, emit in work:
                emit()
            continue
        hc, m = divmod(n, ch)
        base = hc * ch
        work = []
        for i, j, s in ready[hc].get(m, ()):
            work.append((8 + _macc_cost(s), lambda b=base, i=i, j=j, s=s: butterfly(b, i, j, s)))
            if m == ch - 1 and (j - i).bit_length() - 1 == last_q:
                for mm in (i, j):
                    work.append((sum(_macc_cost(c) for _, c in P.acc[(hc, mm)]),
                                 lambda hc=hc, mm=mm: fold(hc, mm)))
        if m == ch - 1 and last_q < 0:        # ch == 1: no butterflies
            work.append((0, lambda hc=hc: fold(hc, 0)))
        if m == ch - 1 and defer and n < k - 1:
            # split by cost into defer + 1 consecutive groups (dependency order kept)
            total = sum(c for c, _ in work)
            groups = [[] for _ in range(defer + 1)]
            acc_c = 0
            for c, emit in work:
                groups[min(defer, int(acc_c * (defer + 1) / max(1, total)))].append(emit)
                acc_c += c
            work = [(0, e) for e in groups.pop(0)]
        elif groups:
            work = [(0, e) for e in groups.pop(0)] + work
        for _, emit in work:
            emit()
    for g in groups:
        for emit in g:
            emit()
    for t in range(P.R):
        if t not in inited:
            for b in range(8):
                E(Op("v_movk", (acc_block(t) + b, 0)))
    for i, j, s in P.final_bfly:
        ei, ej = acc_block(i), acc_block(j)
        if s:
            _macc(E, ei, ej, s, init=False, tmp=tmp)
        for b in range(8):
            E(Op("v_xor", (ej + b, ej + b, ei + b)))


def _prologue(E, spec: KernelSpec):
    E(Op("s_load_args", ()))
    # wave id = workgroup * 4 + (tid >> 6); lane = tid & 63
    E(Op("v_lshr", (V_T, 6, V_LANE)))
    E(Op("v_andk", (V_LANE, 63, V_LANE)))
    E(Op("v_readfirstlane", (29, V_T)))
    if spec.mode == "dec":
        E(Op("s_load_args_dec", ()))
    E(Op("s_load_args_offs", (spec.offs_kernarg,)))
    if spec.mode == "synw":
        E(Op("s_load_karg_x2", (SW_BOUND, KERNARG_BYTES)))   # kernarg words 24..25
    E(Op("s_nop", (4,)))
    E(Op("s_waitcnt_lgkm", ()))
    if spec.merged or spec.head_mark:
        E(Op("label", (".Lhead_end",)))   # _generate_merged: the passes' common head ends here
    if spec.mode == "dec":
        # every wave copies the whole 8 KB split-table set into LDS (no
        # barrier: waves of a workgroup write identical bytes)
        E(Op("s_movk", (62, 4096)))
        E(Op("s_movk", (63, 0)))
        E(Op("v_movs", (V_ADDR, 60)))
        E(Op("v_movs", (V_ADDR + 1, 61)))
        E(Op("v_mad64_k", (V_ADDR, V_LANE, 16, V_ADDR)))
        E(Op("v_add64_s", (V_SRCA, V_ADDR, 62)))
        for q in range(8):
            E(Op("load16", (48 + 4 * q, V_ADDR if q < 4 else V_SRCA, 1024 * (q % 4))))
        # global bytes q*1024 + 16 l = record 32 q + l/2, half l % 2 -> LDS
        # (32 q + l/2) * 256 + 16 (l % 2)
        E(Op("v_lshr", (V_T, 1, V_LANE)))
        E(Op("v_lshl", (V_T, 8, V_T)))
        E(Op("v_andk", (V_T + 1, 1, V_LANE)))
        E(Op("v_lshl", (V_T + 1, 4, V_T + 1)))
        E(Op("v_xor", (V_T, V_T, V_T + 1)))
        for b in range(4):
            E(Op("s_movk", (S_PICK + b, 0x0C0C000C | (b << 8))))
        E(Op("s_waitcnt_vm", (0,)))
        for q in range(8):
            E(Op("ds_write_b128", (V_T, 48 + 4 * q, 32 * LDS_TAB_STRIDE * q)))
        E(Op("s_waitcnt_lgkm_n", (0,)))
    if spec.stagger:
        E(Op("s_stagger", tuple(spec.stagger)))
    if spec.xcd_remap:
        # w' = base(w % 8) + w / 8 with XCD x owning c_x = q + (x < rem)
        # consecutive workgroups, q = nwg / 8, rem = nwg % 8 (a bijection)
        if spec.merged:
            E(Op("s_mov", (46, 18)))         # nwg = the item stride
        else:
            E(Op("s_lshrk", (46, 18, 2)))    # nwg = total waves / 4
        E(Op("s_andk", (47, 2, 7)))          # x
        E(Op("s_lshrk", (30, 46, 3)))        # q
        E(Op("s_mul", (30, 47, 30)))         # x * q
        E(Op("s_andk", (46, 46, 7)))         # rem
        E(Op("s_min", (46, 47, 46)))         # min(x, rem)
        E(Op("s_add", (30, 30, 46)))
        E(Op("s_lshrk", (46, 2, 3)))         # w / 8
        E(Op("s_add", (30, 30, 46)))
        if not spec.merged:
            E(Op("s_lshl", (30, 30, 2)))     # w' * 4
    elif spec.merged:
        E(Op("s_mov", (30, 2)))
    else:
        E(Op("s_lshl", (30, 2, 2)))          # s30 = workgroup_id * 4   (s2 = workgroup id)
    if spec.merged:
        E(Op("s_mov", (28, 30)))             # s28 = the workgroup's item (every pass)
    elif spec.ksplit > 1:
        E(Op("s_lshrk", (28, 30, 2)))        # s28 = the workgroup's item (all its waves)
    else:
        E(Op("s_add", (28, 29, 30)))         # s28 = item = global wave id
    E(Op("s_mov", (32, 10)))
    E(Op("s_movk", (33, 0)))
    E(Op("s_mov", (34, 11)))
    E(Op("s_movk", (35, 0)))
    E(Op("s_movk", (S_ABSENT, ABSENT)))
    if spec.mode == "synw":   # G - 1 = (total - 1) / Lv
        E(Op("s_addk", (SW_GLAST, 14, -1)))
        E(Op("s_mul_hi", (SW_GLAST, SW_GLAST, 15)))
        E(Op("s_lshr_s", (SW_GLAST, SW_GLAST, 16)))
    for q, (_, mask, _) in enumerate(_TRANSPOSE):
        E(Op("s_movk", (S_TMASK + q, mask)))
    if spec.vmask is not None:
        for q in range(3):
            E(Op("v_movs", (spec.vmask[q], S_TMASK + q)))
    E(Op("label", (".Litem",)))
    if spec.far:
        E(Op("s_cmp_lt_br", (28, 17, ".Lgo")))
        E(Op("s_far_jump", (".Lend", 0)))
        E(Op("label", (".Lgo",)))
    else:
        E(Op("s_cmp_ge_br", (28, 17, ".Lend")))
    # unit A = item*128 + lane, unit B = A + 64; valid = unit < total
    for h, (gv, uv, sv, dv, vm, sm) in enumerate(((V_GA, V_UA, V_SRCA, V_DSTA, 26, S_STA),
                                                  (V_GB, V_UB, V_SRCB, V_DSTB, 24, S_STB))):
        if h == 0:
            E(Op("v_lshl_add_s", (V_F, 28, 7, V_LANE)))
        else:
            E(Op("v_addk", (V_F, 64, V_F)))
        E(Op("v_cmp_gt_s", (vm, 14, V_F)))
        # g = mulhi(f, magic) >> shift ; u = f - g*Lu
        E(Op("v_mul_hi_s", (gv, V_F, 15)))
        E(Op("v_lshr_s", (gv, 16, gv)))
        E(Op("v_mul_lo_s", (uv, gv, 13)))
        E(Op("v_sub", (uv, V_F, uv)))
        # load mask: unit in range and u < Lu; store mask: unit in range and
        # (enc) u < s19 / (syn) any u < Lv
        E(Op("v_cmp_gt_s", (S_PAD, 12, uv)))
        if spec.mode == "enc":
            E(Op("v_cmp_gt_s", (S_TMP, 19, uv)))
        E(Op("s_nop", (4,)))
        # (dec: the recovered rows are caller memory -> payload lanes only)
        E(Op("s_and64", (S_TMP2, vm, vm)))   # lanes with a unit (offset-table loads)
        E(Op("s_and64", (sm, vm, {"enc": S_TMP, "syn": vm, "synw": vm, "dec": S_PAD}[spec.mode])))
        E(Op("s_and64", (vm, vm, S_PAD)))
        # src/dst + g * gen_stride + 16 u   (VOP3 reads at most one SGPR), or
        # src/dst + table[g] + 16 u with a generation offset table
        for x, (ptr, base_s, gs_s) in enumerate(((sv, 4, 8), (dv, 6, 9))):
            if spec.mode == "synw" and x == 0:
                E(Op("v_lshl", (sv, 4, uv)))     # synw: the row address is scalar, the lane adds 16 u
                continue
            _gen_base(E, ptr, base_s, gs_s, S_OFFS + 2 * x, gv, S_TMP2, f"{h}{x}")
            E(Op("v_mad64_k", (ptr, uv, 16, ptr)))
        if spec.mode in ("syn", "dec"):
            z = V_ZA if h == 0 else V_ZB
            E(Op("v_movs", (z, 22)))
            E(Op("v_movs", (z + 1, 23)))
            E(Op("v_mad64_k", (z, uv, 16, z)))
    E(Op("s_nop", (4,)))
    E(Op("label", (".Lbody",)))  # marks the end of the per-item setup (tools/bs_lab.py)


def _gen_base(E, ptr: int, base_s: int, gs_s: int, tab_s: int, gv: int, lanes: int, tag: str):
    """ptr <- base + g * gen_stride, or base + table[g] when the table
    pointer s[tab_s:tab_s+1] is non-zero (wave-uniform branch; the table load
    runs on the lanes of `lanes` only, other lanes keep base)."""
    E(Op("v_movs", (ptr, base_s)))
    E(Op("v_movs", (ptr + 1, base_s + 1)))
    E(Op("s_cmp_eq64_0_br", (tab_s, f".Lstrided{tag}")))
    E(Op("v_movs", (V_T, tab_s)))
    E(Op("v_movs", (V_T + 1, tab_s + 1)))
    E(Op("v_mad64_k", (V_T, gv, 8, V_T)))
    E(Op("s_exec", (lanes,)))
    E(Op("load8", (V_T + 2, V_T, 0)))
    E(Op("s_waitcnt_vm", (0,)))
    E(Op("v_add64_v", (ptr, ptr, V_T + 2)))
    E(Op("s_exec", (None,)))
    E(Op("s_branch", (f".Lbased{tag}",)))
    E(Op("label", (f".Lstrided{tag}",)))
    E(Op("v_mad64_s", (ptr, gv, gs_s, ptr)))
    E(Op("label", (f".Lbased{tag}",)))


def _epilogue_next_item(E, far: bool = False):
    E(Op("s_nop", (4,)))  # store data/address VGPRs are rewritten by the next item
    E(Op("s_add", (28, 28, 18)))
    E(Op("s_far_jump", (".Litem", 1)) if far else Op("s_branch", (".Litem",)))
    E(Op("label", (".Lend",)))
    E(Op("s_endpgm", ()))


def valu_per_item(spec: KernelSpec) -> int:
    """VALU instructions one item (one wave's pass over its 128 lane units)
    issues: the ops from the item-loop head to its back-edge.  Exact for the
    encode kernels (straight-line bodies); an upper bound where dec-mode guards
    skip blocks.  bench.py prices the VALU roof of a kernel from it when no SQ
    counter pass of that workload exists (C5 sliding windows).  A merged
    dispatch: the sum over its passes (one wave each per item)."""
    if isinstance(spec, MergedSpec):
        helpers = [dataclasses.replace(spec.passes[0], xchg=(spec.waves, len(spec.passes) + h, True))
                   for h in range(spec.helpers)]
        return sum(valu_per_item(p) for p in list(spec.passes) + helpers)
    ops = generate(spec)
    start = next(n for n, op in enumerate(ops) if op.name == "label" and op.args[0] == ".Litem")
    n = 0
    for op in ops[start + 1:]:
        if op.name in ("s_far_jump", "s_branch") and op.args[0] == ".Litem":
            break
        if op.name.startswith("v_"):
            n += 1
    return n


def generate(spec: KernelSpec) -> list[Op]:
    if isinstance(spec, MergedSpec):
        return _generate_merged(spec)
    if spec.mode == "cmb":
        ops = _generate_cmb(spec)
    elif spec.mode == "enc":
        ops = _generate_enc(spec)
    elif spec.mode == "synw":
        ops = _generate_synw(spec)
    elif spec.mode == "dec" and spec.chunked:
        ops = _generate_dec_chunked(spec)
    else:
        ops = _generate_syn(spec)
    lat = spec.sched or _SCHED_ALL
    if lat:
        from . import bs_sched
        ops = bs_sched.schedule(ops, lat)
    return ops


# tests only: schedule every generated kernel (BS_SCHED_ALL=<slots>), so the
# whole emulator suite checks the scheduler on every kernel family
_SCHED_ALL = int(__import__("os").environ.get("BS_SCHED_ALL", "0") or 0)


@dataclasses.dataclass(frozen=True)
class MergedSpec:
    """Every encode pass of a code with more repairs than one kernel holds, in
    ONE dispatch: a workgroup of len(passes) waves per item, wave p running
    pass p over the item's 128 units.  The passes read the same source rows in
    the same order at about the same time, so all but the first read of each
    row hit the CU's L1 / the XCD's L2 instead of HBM (separate pass launches
    re-read every source row from HBM once per pass)."""
    passes: tuple
    # pass-major: workgroups [p n, (p + 1) n) run pass p over the items as a
    # separate launch of n 4-wave workgroups would (n = s18 / 4), so one pass's
    # last, partly filled round of workgroups overlaps the next pass's first
    concat: bool = False
    # xchg: producer-only waves beside the pass waves (a 3-pass code's
    # workgroup gets a 4th wave that only loads, transposes and transforms
    # row groups, so two workgroups fill a CU's 8 wave slots)
    helpers: int = 0

    chunked = False
    ksplit = 1
    j0 = 0
    far = True

    @property
    def mode(self) -> str:
        return self.passes[0].mode       # "enc" or "synw"

    @property
    def map_stride(self) -> int:
        return self.passes[0].map_stride

    @property
    def k(self) -> int:
        return self.passes[0].k

    @property
    def rt(self) -> int:
        return self.passes[0].rt

    @property
    def r(self) -> int:
        return self.rt

    @property
    def pd(self) -> int:
        return self.passes[0].pd

    @property
    def fft(self) -> int:
        return self.passes[0].fft

    @property
    def waves(self) -> int:
        return 4 if self.concat else len(self.passes) + self.helpers

    @property
    def n_passes(self) -> int:
        return len(self.passes)

    @property
    def name(self) -> str:
        if self.mode == "synw":
            return (f"qf_cauchy_synw{'c' if self.concat else 'm'}{self._xtag}"
                    f"{f'f{self.fft}' if self.fft else ''}_k{self.k}_r{self.rt}")
        return f"qf_cauchy_bsm{self._xtag}{f'f{self.fft}' if self.fft else ''}_k{self.k}_r{self.rt}"

    @property
    def _xtag(self) -> str:
        """'x' for shared row work, 'xh' with producer-only waves."""
        return ("x" + "h" * bool(self.helpers)) if self.passes[0].xchg else ""

    @property
    def next_free_vgpr(self) -> int:
        return max(p.next_free_vgpr for p in self.passes)

    @property
    def next_free_sgpr(self) -> int:
        return max(p.next_free_sgpr for p in self.passes)

    @property
    def kernarg_bytes(self) -> int:
        return self.passes[0].kernarg_bytes

    @property
    def lds_bytes(self) -> int:
        # lds_rows: each wave's row slots at s29 (its pass) x the slots' bytes
        if self.concat or self.passes[0].xchg:
            return max(p.lds_bytes for p in self.passes)
        return self.waves * self.passes[0].lds_rows * LDS_ROW_BYTES


def merged_spec(passes, concat: bool = False, xchg: bool = False, helpers: int = 0) -> MergedSpec:
    assert not (xchg and (concat or passes[0].mode not in ("enc", "synw") or not passes[0].fft or passes[0].lds_rows))
    assert not helpers or xchg
    if xchg:   # the waves share the groups: every pass streams the same rows through the same chunk transforms
        g0 = [(rows, bf) for rows, bf, _ in xchg_groups(passes[0].fplan)]
        assert all([(rows, bf) for rows, bf, _ in xchg_groups(p.fplan)] == g0 for p in passes[1:])
    nw = len(passes) + helpers
    passes = tuple(dataclasses.replace(p, merged=not concat, head_mark=concat,
                                       xchg=(nw, n) if xchg else ()) for n, p in enumerate(passes))
    assert 1 < len(passes) <= 16 and all(p.mode == passes[0].mode in ("enc", "synw") and p.ksplit == 1
                                        for p in passes)
    assert len({p.lds_rows for p in passes}) == 1 and (not passes[0].lds_rows or passes[0].fft)
    assert all(p.k == passes[0].k and p.rt == passes[0].rt for p in passes)
    assert sorted((p.j0, p.j0 + p.r) for p in passes) == [(p.j0, p.j0 + p.r) for p in passes]
    assert passes[0].j0 == 0 and passes[-1].j0 + passes[-1].r == passes[0].rt
    return MergedSpec(passes, concat, helpers)


def _generate_merged(ms: MergedSpec) -> list[Op]:
    """The common head (kernargs, lane / wave ids), a branch on the wave's
    index in its workgroup (s29) to its pass, and each pass's body (its own
    item loop, labels and far-jump ids made unique).  A pass's body first
    moves the output base s[6:7] to its first row: + j0 * output row stride
    (repair rows for enc, syndrome rows for synw)."""
    out: list[Op] = []
    E = out.append
    bodies = []
    streams = list(ms.passes) + [dataclasses.replace(ms.passes[0], xchg=(ms.waves, len(ms.passes) + h, True))
                                 for h in range(ms.helpers)]
    for p, sp in enumerate(streams):
        ops = generate(sp)
        cut = next(n for n, op in enumerate(ops) if op.name == "label" and op.args[0] == ".Lhead_end")
        if p == 0:
            out.extend(ops[:cut])
        bodies.append(ops[cut + 1:])
    if ms.concat:
        # pass p = the workgroup id's range; s2 becomes the id within it
        E(Op("s_lshrk", (46, 18, 2)))            # n = workgroups per pass
        for p in range(ms.n_passes - 1):
            E(Op("s_cmp_lt_br", (2, 46, f".Lsel{p}")))
            E(Op("s_sub", (2, 2, 46)))
        E(Op("s_far_jump", (f".Lpass{ms.n_passes - 1}", 900)))
        for p in range(ms.n_passes - 1):
            E(Op("label", (f".Lsel{p}",)))
            E(Op("s_far_jump", (f".Lpass{p}", 901 + p)))
    else:
        for p in range(1, ms.waves):
            E(Op("s_cmp_lg_k_br", (29, p, f".Lnpass{p}")))
            E(Op("s_far_jump", (f".Lpass{p}", 900 + p)))
            E(Op("label", (f".Lnpass{p}",)))
    for p, body in enumerate(bodies):
        E(Op("label", (f".Lpass{p}",)))
        j0 = ms.passes[p].j0 if p < len(ms.passes) else 0
        if j0:
            E(Op("s_mul_k", (46, 11, j0)))
            E(Op("s_add", (6, 6, 46)))
            E(Op("s_addck", (7, 7, 0)))
        for op in body:
            args = tuple(a.replace(".L", f".LP{p}", 1) if isinstance(a, str) and a.startswith(".L") else a
                         for a in op.args)
            if op.name == "s_far_jump":
                args = (args[0], args[1] + 1000 * (p + 1))
            E(Op(op.name, args))
    return out


def _store_pair(E, acc: int, ma: int, mb: int, pol: str = ""):
    E(Op("s_exec", (ma,)))
    E(Op("store16", (V_DSTA, acc, 0, pol)))
    E(Op("s_exec", (mb,)))
    E(Op("store16", (V_DSTB, acc + 4, 0, pol)))
    E(Op("s_exec", (None,)))
    E(Op("v_add64_s", (V_DSTA, V_DSTA, 34)))
    E(Op("v_add64_s", (V_DSTB, V_DSTB, 34)))


def _generate_enc(spec: KernelSpec) -> list[Op]:
    if spec.xchg:
        return _generate_xchg(spec)
    k, r, pd, nbuf = spec.k, spec.r, spec.pd, spec.nbuf
    assert spec.j0 + r <= spec.rt
    C = cauchy(k, spec.rt)[spec.j0: spec.j0 + r]
    acc0, ring0 = spec.acc0, spec.ring0
    ops: list[Op] = []
    E = ops.append
    _prologue(E, spec)

    ks = spec.ksplit
    step = 46 if ks > 1 else 32       # row pointer step: s[46:47] = {ks * row stride, 0}

    def load_row(row: int):
        b = ring0 + 8 * (row % nbuf)
        E(Op("s_exec", (26,)))
        E(Op("load16", (b, V_SRCA, 0, spec.ld_policy)))
        E(Op("s_exec", (24,)))
        E(Op("load16", (b + 4, V_SRCB, 0, spec.ld_policy)))
        E(Op("s_exec", (None,)))
        E(Op("v_add64_s", (V_SRCA, V_SRCA, step)))
        E(Op("v_add64_s", (V_SRCB, V_SRCB, step)))

    if spec.fft:
        assert ks == 1
        cur = [0]      # source row the row pointers address
        S = spec.lds_rows
        v_ldsa = spec.next_free_vgpr - 1 if S else None

        def load_fft(n: int, base: int):
            i = spec.fplan.order[n]
            if i != cur[0]:
                E(Op("s_mul_k", (46, 10, i - cur[0])))     # (i - cur) * row stride, signed
                E(Op("s_ashr31", (47, 46)))
                E(Op("v_add64_s", (V_SRCA, V_SRCA, 46)))
                E(Op("v_add64_s", (V_SRCB, V_SRCB, 46)))
                cur[0] = i
            for h, (vm, va) in enumerate(((26, V_SRCA), (24, V_SRCB))):
                E(Op("s_exec", (vm,)))
                if S:
                    E(Op("s_m0", (S_ROWLDS_ENC, (n % S) * LDS_ROW_BYTES + 1024 * h)))
                    E(Op("load16_lds", (va, spec.ld_policy)))
                else:
                    E(Op("load16", (base + 4 * h, va, 0, spec.ld_policy)))
            E(Op("s_exec", (None,)))

        def wait_fft(n: int):
            E(Op("s_waitcnt_vm", (2 * min(spec.ahead, k - 1 - n),)))
            if S:
                base = ring0 + 8 * (n % spec.nbuf)
                E(Op("ds_read_b128", (base, v_ldsa, (n % S) * LDS_ROW_BYTES)))
                E(Op("ds_read_b128", (base + 4, v_ldsa, (n % S) * LDS_ROW_BYTES + 1024)))
                E(Op("s_waitcnt_lgkm_n", (0,)))

        if S:   # this wave's LDS row slots (lds_rows x 2 KiB per wave) and its ds_read address
            E(Op("s_movk", (S_ROWLDS_ENC, S * LDS_ROW_BYTES)))
            E(Op("s_mul", (S_ROWLDS_ENC, S_ROWLDS_ENC, 29)))
            E(Op("v_lshl", (v_ldsa, 4, V_LANE)))
            E(Op("v_add_s", (v_ldsa, S_ROWLDS_ENC, v_ldsa)))
        _fft_stream(E, ops, spec, load_fft, wait_fft, lambda t: acc0 + 8 * t)

    def rows_of(srcs: list[int]):
        for m in range(min(pd, len(srcs))):
            load_row(m)
        for m, i in enumerate(srcs):
            if m + pd < len(srcs):
                load_row(m + pd)
            after = min(pd, len(srcs) - 1 - m)
            E(Op("s_waitcnt_vm", (2 * after,)))
            _source_row(ops, C, i, r, ring0 + 8 * (m % nbuf), acc0, init=(m == 0), xor3=spec.xor3,
                        bfi=spec.bfi_transpose, vmask=spec.vmask)

    if ks > 1:
        # wave w: sources w, w + ks, ... (k >= ks): start at row w, step ks rows
        assert k >= ks
        E(Op("s_mul", (46, 29, 10)))
        E(Op("s_movk", (47, 0)))
        E(Op("v_add64_s", (V_SRCA, V_SRCA, 46)))
        E(Op("v_add64_s", (V_SRCB, V_SRCB, 46)))
        E(Op("s_movk", (46, ks)))
        E(Op("s_mul", (46, 46, 10)))
        for w in range(1, ks):
            E(Op("s_cmp_lg_k_br", (29, w, f".Lnsec{w}")))
            E(Op("s_far_jump", (f".Lsec{w}", 40 + w)))
            E(Op("label", (f".Lnsec{w}",)))
        for w in range(ks):
            E(Op("label", (f".Lsec{w}",)))
            rows_of([i for i in range(k) if i % ks == w])
            if w + 1 < ks:
                E(Op("s_far_jump", (".Lsec_end", 50 + w)))
        E(Op("label", (".Lsec_end",)))
    elif not spec.fft:
        rows_of(list(range(k)))
    # accumulator block of repair j
    blk = (lambda j: acc0 + 8 * spec.fplan.out_block[j]) if spec.fft else (lambda j: acc0 + 8 * j)
    # planes -> bytes, store 2 x 16 bytes per lane per repair
    for j in range(r):
        ops.extend(_transpose_ops(blk(j), spec.bfi_transpose, spec.vmask))
    if ks > 1:   # partial repairs of waves 1.. into wave 0 (temps: the ring, dead now)
        _ksplit_reduce(E, ks, r, acc0, ring0, ring0 + 8, 0, jmax_guard=False)
    _enc_store_repairs(E, spec, blk)
    if ks > 1:
        _ksplit_epilogue(E)
    else:
        _epilogue_next_item(E, far=spec.far)
    return ops


def xchg_groups(P) -> list[tuple[list[int], list, list]]:
    """The row groups of an additive-FFT pass plan, in fold order: every
    chunk (plan rows hc*ch .. hc*ch + ch - 1, its inverse butterflies, each
    row's accumulator constants) and then the rows that enter directly (no
    butterflies).  The groups depend on the plan's source side only, the
    constants on the pass."""
    ch = P.ch
    kA = getattr(P, "kA", 0) or P.k
    groups = [(list(range(hc * ch, hc * ch + ch)), P.chunk_bfly[hc], [P.acc[(hc, m)] for m in range(ch)])
              for hc in range(kA // ch)]
    direct = sorted(getattr(P, "direct", {}))
    for q in range(0, len(direct), ch):
        rows = direct[q: q + ch]
        groups.append((rows, [], [P.direct[n] for n in rows]))
    return groups


def _generate_xchg(spec: KernelSpec) -> list[Op]:
    """One wave's stream of a merged additive-FFT encode (or synw) whose waves share
    the row work (MergedSpec with xchg).  Every pass of a code streams the
    same source rows through the same chunk transforms (xchg_groups: only the
    fold constants and the final butterflies depend on the pass), so wave w of
    the workgroup loads, transposes and inverse-transforms only the groups
    n * W + w (round n, W waves) and writes their planes to its LDS slot;
    after a barrier every wave folds the round's W groups from LDS into its
    own pass's accumulators, and a second barrier frees the slots.  Per wave
    that is 1/W of the loads, transposes and chunk butterflies (58 % of a
    (196, 59) pass's VALU before) and 1/W of the code they take.  The loads of
    a wave's next group are issued as soon as its planes are in LDS, so they
    fly during the fold phase; with spec.xchg_early its first rows already
    before the transform, into 8-VGPR row slots the current group does not
    hold (the slots rotate roles).  Every stream has the same barrier sequence
    and item loop, so the workgroup's waves meet at every barrier.

    synw (decode syndromes, slot-map gather): the groups' rows are the
    received sources (the zero row where absent), the pass's accepted repairs
    are XORed onto its syndromes in byte form at the end (their loads issued
    once the wave's last group is in LDS), and a wave whose pass no
    generation of the item needs (s[SW_SKIP]) still produces its groups but
    skips its folds and stores.  A producer-only wave (spec.xchg[2],
    MergedSpec.helpers) produces its share of the groups and folds nothing."""
    synw = spec.mode == "synw"
    nw, me = spec.xchg[:2]
    helper = len(spec.xchg) > 2 and spec.xchg[2]   # a producer-only wave (no pass of its own)
    P = spec.fplan
    ch = P.ch
    ring0, acc0 = spec.ring0, spec.acc0
    nslot = spec.nbuf                    # 8-VGPR row slots from ring0 (rotating roles)
    early = spec.xchg_early
    v_ldsa = spec.next_free_vgpr - 1
    tmp = tuple(range(V_T, V_T + 4)) if spec.fft_cse else ()
    groups = xchg_groups(P)
    G = len(groups)
    nrounds = -(-G // nw)
    slot_bytes = ch * LDS_ROW_BYTES
    assert nw * slot_bytes <= 65536 and all(len(g[0]) <= ch for g in groups)
    ops: list[Op] = []
    E = ops.append
    _prologue(E, spec)
    if synw:
        _synw_item_setup(E, spec)
    E(Op("v_lshl", (v_ldsa, 4, V_LANE)))      # LDS byte offset of the lane's 16-B unit A
    cur = [0]            # source row the row pointers address (row 0 after the item setup)
    quad = [None]        # synw: the slot-map quad in s[SW_Q0..] / s[SW_Q1..]

    def slot(x: int) -> int:
        return ring0 + 8 * x

    def load_group(gi: int, ms=None, slots=None):
        rows = groups[gi][0]
        ms = range(len(rows)) if ms is None else ms
        for m in ms:
            n = rows[m]
            base = slot(slots[m]) if slots is not None else ring0 + 8 * m
            if synw:
                _synw_load_row(E, spec, quad, "src", P.order[n], base)
                continue
            i = P.order[n]
            if i != cur[0]:
                E(Op("s_mul_k", (46, 10, i - cur[0])))     # (i - cur) * row stride, signed
                E(Op("s_ashr31", (47, 46)))
                E(Op("v_add64_s", (V_SRCA, V_SRCA, 46)))
                E(Op("v_add64_s", (V_SRCB, V_SRCB, 46)))
                cur[0] = i
            for h, (vm, va) in enumerate(((26, V_SRCA), (24, V_SRCB))):
                E(Op("s_exec", (vm,)))
                E(Op("load16", (base + 4 * h, va, 0, spec.ld_policy)))
            E(Op("s_exec", (None,)))

    per_row = (0 if spec.lab_norows else 4) if synw else 2    # loads per row

    def produce(gi: int, rs: list, nxt):
        """Transform group gi, whose row m sits in slot rs[m], and write it to
        LDS; nxt = (group, slots) of the wave's next group: its first `early`
        rows load before the transform (into slots rs does not hold), the rest
        after it.  Returns the next group's slots by row."""
        rows, bfly, _ = groups[gi]
        ne = min(early, len(groups[nxt][0])) if nxt is not None else 0
        nslots = None
        if nxt is not None:
            nslots = [None] * len(groups[nxt][0])
            free = [x for x in range(nslot) if x not in rs]
            for m in range(ne):
                nslots[m] = free[m]
            load_group(nxt, range(ne), nslots)
        E(Op("s_waitcnt_vm", (per_row * ne,)))
        for m in range(len(rows)):
            ops.extend(_transpose_ops(slot(rs[m]), spec.bfi_transpose, spec.vmask))
        for i, j, c in bfly:           # y_j ^= y_i; y_i ^= c y_j (lch_fft.Plan.chunk_bfly)
            yi, yj = slot(rs[i]), slot(rs[j])
            for b in range(8):
                E(Op("v_xor", (yj + b, yj + b, yi + b)))
            if c:
                _macc(E, yi, yj, c, init=False, tmp=tmp)
        for m in range(len(rows)):
            off = me * slot_bytes + m * LDS_ROW_BYTES
            E(Op("ds_write_b128", (v_ldsa, slot(rs[m]), off)))
            E(Op("ds_write_b128", (v_ldsa, slot(rs[m]) + 4, off + 1024)))
        E(Op("s_waitcnt_lgkm_n", (0,)))      # planes in LDS; their slots are free
        if nxt is not None and ne < len(nslots):
            free = [x for x in range(nslot) if x not in nslots[:ne]]
            for m in range(ne, len(nslots)):
                nslots[m] = free[m - ne]
            load_group(nxt, range(ne, len(nslots)), nslots)
        return nslots

    inited: set = set()

    def consume(rnd: int, busy: list):
        # the two read-back buffers: slots no pending load targets
        bufs = [x for x in reversed(range(nslot)) if x not in busy][:2]
        rowbuf = (slot(bufs[0]), slot(bufs[1]))
        seq = [(q, m) for q in range(nw) if rnd * nw + q < G for m in range(len(groups[rnd * nw + q][0]))]
        if synw:
            E(Op("s_cmp_lg_k_br", (SW_SKIP, 0, f".Lnofold{rnd}")))

        def read(x: int):
            q, m = seq[x]
            buf = rowbuf[x % 2]
            off = q * slot_bytes + m * LDS_ROW_BYTES
            E(Op("ds_read_b128", (buf, v_ldsa, off)))
            E(Op("ds_read_b128", (buf + 4, v_ldsa, off + 1024)))
        read(0)
        for x, (q, m) in enumerate(seq):
            if x + 1 < len(seq):
                read(x + 1)
                E(Op("s_waitcnt_lgkm_n", (2,)))
            else:
                E(Op("s_waitcnt_lgkm_n", (0,)))
            for t, c in groups[rnd * nw + q][2][m]:
                _macc(E, acc0 + 8 * t, rowbuf[x % 2], c, init=t not in inited, tmp=tmp)
                inited.add(t)
        if synw:
            E(Op("label", (f".Lnofold{rnd}",)))

    issued: list = []     # synw: repair rows in load order (per_row loads each)

    def load_repair(j: int):
        _synw_load_row(E, spec, quad, "rep", j, ring0 + 8 * (j % ch))
        issued.append(j)

    def mine(rnd: int):
        gi = rnd * nw + me
        return gi if gi < G else None

    rs = None           # slots of the wave's current group, by row
    if mine(0) is not None:
        rs = list(range(len(groups[mine(0)][0])))
        load_group(mine(0), None, rs)
    elif synw and not helper:
        for j in range(min(ch, spec.r)):
            load_repair(j)
    busy = list(rs or []) + (list(range(min(ch, spec.r))) if issued else [])
    for rnd in range(nrounds):
        gi = mine(rnd)
        if gi is not None:
            rs = produce(gi, rs, mine(rnd + 1))
            busy = list(rs or [])
            if rs is None and synw and not helper:    # the wave's last group: slots 0.. take the first repairs
                for j in range(min(ch, spec.r)):
                    load_repair(j)
                busy = list(range(min(ch, spec.r)))
        E(Op("s_barrier", ()))
        if not helper:
            consume(rnd, busy)
        E(Op("s_barrier", ()))
    if helper:
        if synw:
            E(Op("label", (".Lskip",)))
        _epilogue_next_item(E, far=spec.far)
        return ops
    if synw:
        E(Op("s_cmp_eq_k_br", (SW_SKIP, 0, ".Lfold_all")))
        E(Op("s_waitcnt_vm", (0,)))
        E(Op("s_far_jump", (".Lskip", 3)))
        E(Op("label", (".Lfold_all",)))
    for t in range(P.R):
        if t not in inited:
            for b in range(8):
                E(Op("v_movk", (acc0 + 8 * t + b, 0)))
    for i, j, c in P.final_bfly:
        ei, ej = acc0 + 8 * i, acc0 + 8 * j
        if c:
            _macc(E, ei, ej, c, init=False, tmp=tmp)
        for b in range(8):
            E(Op("v_xor", (ej + b, ej + b, ei + b)))

    def blk(j):
        return acc0 + 8 * P.out_block[j]
    for j in range(spec.r):
        ops.extend(_transpose_ops(blk(j), spec.bfi_transpose, spec.vmask))
        if synw:      # + the accepted repair (byte form); its registers then take repair j + ch
            E(Op("s_waitcnt_vm", (per_row * (len(issued) - 1 - issued.index(j)),)))
            base = ring0 + 8 * (j % ch)
            for b in range(8):
                E(Op("v_xor", (blk(j) + b, blk(j) + b, base + b)))
            if j + ch < spec.r:
                load_repair(j + ch)
    if synw:
        E(Op("s_nop", (4,)))
        for j in range(spec.r):
            _store_pair(E, blk(j), S_STA, S_STB, spec.st_policy)
        E(Op("label", (".Lskip",)))
    else:
        _enc_store_repairs(E, spec, blk)
    _epilogue_next_item(E, far=spec.far)
    return ops


def _enc_store_repairs(E, spec: KernelSpec, blk):
    """The repairs (byte form in the accumulator blocks blk(j)) to memory:
    padding lanes zeroed, the partial last unit masked, 2 x 16 B per lane."""
    r = spec.r
    # padding lanes (stored, not loaded: the zero tail) hold garbage, since
    # masked loads leave stale planes in their half of the ring; byte
    # positions are independent, so clearing their half of the repairs here
    # is enough
    for h, (vm, sm) in enumerate(((26, S_STA), (24, S_STB))):
        E(Op("s_andn2_64", (S_PAD, sm, vm)))
        E(Op("s_exec", (S_PAD,)))
        for j in range(r):
            for q in range(4):
                E(Op("v_movk", (blk(j) + 4 * h + q, 0)))
    # the row's last unit when L % 16 != 0 (zero tail only): its bytes >= L
    # come from the source rows' padding; AND them away with the per-dword
    # byte masks s20..s23 (all ones when L % 16 == 0)
    E(Op("s_exec", (None,)))
    E(Op("s_cmp_eq_k_br", (23, MASK32, ".Ltail1")))   # L % 16 == 0: no partial unit
    for h, (uv, sm) in enumerate(((V_UA, S_STA), (V_UB, S_STB))):
        E(Op("s_exec", (None,)))
        E(Op("v_addk", (V_T, 1, uv)))
        E(Op("v_cmp_eq_s", (S_PAD, 12, V_T)))     # u + 1 == Lu
        E(Op("s_nop", (4,)))
        E(Op("s_and64", (S_PAD, S_PAD, sm)))
        E(Op("s_exec", (S_PAD,)))
        E(Op("s_cbranch_execz", (f".Ltail{h}",)))
        for j in range(r):
            for q in range(4):
                x = blk(j) + 4 * h + q
                E(Op("v_and_s", (x, 20 + q, x)))
        E(Op("label", (f".Ltail{h}",)))
    E(Op("s_exec", (None,)))
    E(Op("s_nop", (4,)))
    for j in range(r):
        _store_pair(E, blk(j), S_STA, S_STB, spec.st_policy)


def _jmax(E, k: int, r: int, present):
    """s[S_JMAX] <- 1 + the largest repair index accepted by any lane (both
    halves, payload lanes), 0 if none."""
    for j in reversed(range(r)):
        present(k + j, 0, S_TMP)
        E(Op("s_and64", (S_TMP, S_TMP, S_STA)))
        present(k + j, 1, S_TMP2)
        E(Op("s_and64", (S_TMP2, S_TMP2, S_STB)))
        E(Op("s_or64", (S_TMP, S_TMP, S_TMP2)))
        E(Op("s_movk", (S_JMAX, j + 1)))
        E(Op("s_cmp_lg64_br", (S_TMP, ".Ljdone")))
    E(Op("s_movk", (S_JMAX, 0)))
    E(Op("label", (".Ljdone",)))


def _lu_solve_and_store(E, spec: KernelSpec):
    """Decode stage B in registers: per half, solve C[J, E] x = s in place on
    the syndrome blocks by the packed LU record of the half's generation
    (written by k_decode_prepare_cauchy with lu_out), then store block t to
    recovered row rank[t] of its generation.

    Blocks are the repair indices t < r; the record embeds the e x e LU of
    C[J, E] (J accepted repairs ascending, E erased sources ascending) into
    a 16 x 16 byte matrix, column u at byte 16u: byte t < u =
    U'[t][u] = U[t][u] / U[t][t], byte u = 1 / U[u][u], byte t > u = L[t][u]
    (0 where t or u is not accepted), then rank[t] at byte 256 + t (0xFF:
    not accepted).  Forward: y_t ^= L[t][u] y_u (t > u) and y_u /= U[u][u]
    with the same selectors of y_u; backward: x_t ^= U'[t][u] x_u (t < u).
    Multiplication by a per-lane coefficient c uses the split tables of
    gf256_tables.h from LDS: c * x = T0[x & 7] ^ T1[x >> 3 & 7] ^ T2[x >> 6]
    with v_perm_b32 (four byte lookups per instruction).  The 17 record
    loads of a half are issued together; table reads run one coefficient
    ahead of the v_perm work (two table buffers)."""
    r, acc0 = spec.r, spec.acc0
    masks = (S_STA, S_STB)
    gvs = (V_GA, V_GB)
    R_COLS, R_RANK = lu_layout(spec)
    lu = spec.lu
    # store address pairs in the (then dead) column slots
    st_addr = [c + 2 * q for c in R_COLS for q in range(2)]

    def blk(t, h, d):
        return acc0 + 8 * t + 4 * h + d

    def col(u):
        return R_COLS[u]

    def selectors(u, h):
        for d in range(4):
            x = blk(u, h, d)
            E(Op("v_andk", (R_SEL + d, 0x07070707, x)))
            E(Op("v_lshr", (R_SEL + 4 + d, 3, x)))
            E(Op("v_andk", (R_SEL + 4 + d, 0x07070707, R_SEL + 4 + d)))
            E(Op("v_lshr", (R_SEL + 8 + d, 6, x)))
            E(Op("v_andk", (R_SEL + 8 + d, 0x03030303, R_SEL + 8 + d)))

    def table_read(u, byte, buf):
        a, tb = R_TA[buf], R_TB[buf]
        E(Op("v_perm_s", (a, col(u) + byte // 4, col(u) + byte // 4, S_PICK + byte % 4)))
        E(Op("ds_read_b128", (tb, a, 0)))
        E(Op("ds_read_b32", (tb + 4, a, 16)))

    def products(d, buf):
        tb = R_TB[buf]
        E(Op("v_perm", (R_P, tb + 1, tb, R_SEL + d)))
        E(Op("v_perm", (R_P + 1, tb + 3, tb + 2, R_SEL + 4 + d)))
        E(Op("v_perm", (R_P + 2, tb + 4, tb + 4, R_SEL + 8 + d)))

    def mul_acc(t, h, buf):
        for d in range(4):
            products(d, buf)
            E(Op("v_xor3", (blk(t, h, d), blk(t, h, d), R_P, R_P + 1)))
            E(Op("v_xor", (blk(t, h, d), blk(t, h, d), R_P + 2)))

    def scale(u, h, buf):
        for d in range(4):
            products(d, buf)
            E(Op("v_xor3", (blk(u, h, d), R_P, R_P + 1, R_P + 2)))

    def column(u, h, steps, end_label, guard_from):
        """steps: [(kind, t)] with kind "acc" (block t ^= c_t x_u) or "scale"
        (block u = c_u y_u, then the selectors of x_u); c_t = byte t of
        column u.  Steps at index >= guard_from stop the column (jump to
        end_label) once t >= jmax."""
        table_read(u, steps[0][1], 0)
        for n, (kind, t) in enumerate(steps):
            buf = n % 2
            if n + 1 < len(steps):
                table_read(u, steps[n + 1][1], 1 - buf)
                E(Op("s_waitcnt_lgkm_n", (2,)))
            else:
                E(Op("s_waitcnt_lgkm_n", (0,)))
            if kind == "acc":
                mul_acc(t, h, buf)
            else:
                scale(u, h, buf)   # y_u /= U[u][u]; the selectors still hold y_u
            if n + 1 < len(steps) and n + 1 >= guard_from:
                E(Op("s_cmp_le_k_br", (S_JMAX, steps[n + 1][1], end_label)))
        E(Op("label", (end_label,)))
        E(Op("s_waitcnt_lgkm_n", (0,)))

    for h in range(2):
        E(Op("v_movs", (R_FP, 56)))
        E(Op("v_movs", (R_FP + 1, 57)))
        E(Op("v_mad64_s", (R_FP, gvs[h], 58, R_FP)))
        E(Op("s_exec", (masks[h],)))
        for u in range(r if lu else 0):
            E(Op("load16", (col(u), R_FP, 16 * u)))
        E(Op("load16", (R_RANK[h], R_FP, 256)))
        E(Op("s_exec", (None,)))
        if not lu:
            E(Op("s_waitcnt_vm", (0,)))
            continue
        # forward substitution with unit-lower L, column by column; each
        # final y_u is divided by its pivot with the same selectors
        for u in range(r):
            E(Op("s_cmp_le_k_br", (S_JMAX, u, f".Lfwd_end{h}")))
            E(Op("s_waitcnt_vm", (r - u,)))      # column u (and the ones before) landed
            selectors(u, h)
            column(u, h, [("scale", u)] + [("acc", t) for t in range(u + 1, r)], f".Lfwd{u}_{h}", 1)
        E(Op("label", (f".Lfwd_end{h}",)))
        E(Op("s_waitcnt_vm", (0,)))
        # backward substitution with unit-upper U': y_t ^= U'[t][u] x_u, t < u
        for u in reversed(range(1, r)):
            E(Op("s_cmp_le_k_br", (S_JMAX, u, f".Lbwd{u}_{h}")))
            selectors(u, h)
            column(u, h, [("acc", t) for t in range(u)], f".Lbwd{u}_{h}", r + 1)
    # stores: block t of half h -> recovered row rank[t] of the half's generation
    E(Op("s_nop", (4,)))
    na = 0
    for t in range(r):
        E(Op("s_cmp_le_k_br", (S_JMAX, t, ".Lst_end")))
        for h in range(2):
            rk = R_RANK[h]
            a = st_addr[na % len(st_addr)]
            na += 1
            E(Op("v_bfe", (V_SLOT, rk + t // 4, 8 * (t % 4), 8)))
            E(Op("v_cmp_ne_s", (S_TMP, S_ABSENT, V_SLOT)))
            E(Op("s_nop", (4,)))
            E(Op("s_and64", (S_TMP, S_TMP, masks[h])))
            E(Op("v_mad64_s", (a, V_SLOT, 11, V_DSTA if h == 0 else V_DSTB)))
            E(Op("s_exec", (S_TMP,)))
            E(Op("store16", (a, blk(t, h, 0), 0, spec.st_policy)))
            E(Op("s_exec", (None,)))
    E(Op("label", (".Lst_end",)))


def _generate_syn(spec: KernelSpec) -> list[Op]:
    """Decode stage A: syndromes s_j = p_j ^ sum_{i present} C[j][i] x_i of
    every accepted repair j, for the generation of each half-lane.

    The slot map (per generation: k source slots then r repair slots, one
    byte each, ABSENT if the row was not accepted) says where each row sits
    among the received rows.  Rows stream through the ring in the order
    repairs 0..r-1 (which initialise the accumulators), sources 0..k-1; a
    half whose generation lacks a row reads the zero row instead.
    Syndromes are stored only for accepted repairs."""
    k, r, pd, nbuf = spec.k, spec.r, spec.pd, spec.nbuf
    C = cauchy(k, r)
    acc0, ring0 = spec.acc0, spec.ring0
    maps = (spec.map_a, spec.map_b)
    dec = spec.mode == "dec"
    # dec: sources first (row 0 initialises the accumulators), then the
    # repairs, each XORed in byte form right after its block is transposed
    # back (no transpose of the repair rows themselves)
    if dec:
        seq = [("src", i) for i in range(k)] + [("rep", j) for j in range(r)]
    else:
        seq = [("rep", j) for j in range(r)] + [("src", i) for i in range(k)]
    ops: list[Op] = []
    E = ops.append
    _prologue(E, spec)
    # slot maps of both halves' generations
    # (store masks: padding lanes read their generation's map too, so they
    # store only the accepted repairs' rows, like the payload lanes)
    for h, (gv, vm) in enumerate(((V_GA, S_STA), (V_GB, S_STB))):
        E(Op("v_movs", (V_ADDR, 20)))
        E(Op("v_movs", (V_ADDR + 1, 21)))
        E(Op("v_mad64_s", (V_ADDR, gv, 19, V_ADDR)))
        E(Op("s_exec", (vm,)))
        for q in range(spec.map_quads):
            E(Op("load16", (maps[h] + 4 * q, V_ADDR, 16 * q)))
        E(Op("s_exec", (None,)))
    E(Op("s_waitcnt_vm", (0,)))

    def map_byte(entry) -> int:
        kind, idx = entry
        return idx if kind == "src" else k + idx

    def present(pos: int, h: int, sm: int):
        """v_slot <- slot byte of half h, s[sm] <- slot != ABSENT."""
        E(Op("v_bfe", (V_SLOT, maps[h] + pos // 4, 8 * (pos % 4), 8)))
        E(Op("v_cmp_ne_s", (sm, S_ABSENT, V_SLOT)))
        E(Op("s_nop", (4,)))

    def load_row(n: int):
        b = ring0 + 8 * (n % nbuf)
        pos = map_byte(seq[n])
        for h, (base, z, vm) in enumerate(((V_SRCA, V_ZA, 26), (V_SRCB, V_ZB, 24))):
            present(pos, h, S_TMP)
            E(Op("v_mad64_s", (V_ADDR, V_SLOT, 10, base)))
            E(Op("v_cndmask", (V_ADDR, z, V_ADDR, S_TMP)))
            E(Op("v_cndmask", (V_ADDR + 1, z + 1, V_ADDR + 1, S_TMP)))
            E(Op("s_exec", (vm,)))
            if not spec.lab_norows:
                E(Op("load16", (b + 4 * h, V_ADDR, 0, spec.ld_policy)))
            E(Op("s_exec", (None,)))

    if dec:
        _jmax(E, k, r, present)
        if spec.prio != (0, 0):
            E(Op("s_setprio", (spec.prio[0],)))
    g0 = spec.guard_min
    n_seq = len(seq)
    for n in range(min(pd, n_seq)):
        load_row(n)
    for n, (kind, idx) in enumerate(seq):
        if n + pd < n_seq:
            load_row(n + pd)
        after = min(pd, n_seq - 1 - n)
        E(Op("s_waitcnt_vm", (0 if spec.lab_norows else 2 * after,)))
        base = ring0 + 8 * (n % nbuf)
        if kind == "rep" and dec:
            E(Op("s_cmp_le_k_br", (S_JMAX, idx, f".Lrep{idx}")))
            ops.extend(_transpose_ops(acc0 + 8 * idx, spec.bfi_transpose, spec.vmask))
            for b in range(8):
                E(Op("v_xor", (acc0 + 8 * idx + b, acc0 + 8 * idx + b, base + b)))
            E(Op("label", (f".Lrep{idx}",)))
        elif kind == "rep":
            ops.extend(_transpose_ops(base, spec.bfi_transpose, spec.vmask))
            for b in range(8):
                E(Op("v_mov", (acc0 + 8 * idx + b, base + b)))
        else:
            _source_row(ops, C, idx, r, base, acc0, init=dec and idx == 0, xor3=spec.xor3,
                        bfi=spec.bfi_transpose, vmask=spec.vmask, guard=(g0, f".Lrow{n}") if dec else None)
    if dec:
        if spec.prio != (0, 0):
            E(Op("s_setprio", (spec.prio[1],)))
        _lu_solve_and_store(E, spec)
        _epilogue_next_item(E, far=True)
        return ops
    for j in range(r):
        ops.extend(_transpose_ops(acc0 + 8 * j, spec.bfi_transpose, spec.vmask))
    E(Op("s_nop", (4,)))
    for j in range(r):
        present(k + j, 0, S_TMP)
        E(Op("s_and64", (S_TMP, S_TMP, S_STA)))
        present(k + j, 1, S_TMP2)
        E(Op("s_and64", (S_TMP2, S_TMP2, S_STB)))
        _store_pair(E, acc0 + 8 * j, S_TMP, S_TMP2, spec.st_policy)
    _epilogue_next_item(E, far=spec.far)
    return ops


def _scalar_gen_base(E, dst: int, base_s: int, gs_s: int, tab_s: int, g: int, tag: str):
    """s[dst:dst+1] <- s[base_s:+1] + g * s[gs_s], or + table[g] when the
    64-bit table pointer s[tab_s:tab_s+1] is non-zero (scalar unit)."""
    E(Op("s_cmp_eq64_0_br", (tab_s, f".Lsgs{tag}")))
    E(Op("s_lshl", (SW_T0, g, 3)))
    E(Op("s_lshrk", (SW_T1, g, 29)))
    E(Op("s_add_cc", (SW_T0, SW_T0, tab_s)))
    E(Op("s_addc", (SW_T1, SW_T1, tab_s + 1)))
    E(Op("s_load_x2", (dst, SW_T0, 0)))
    E(Op("s_waitcnt_lgkm", ()))
    E(Op("s_add_cc", (dst, dst, base_s)))
    E(Op("s_addc", (dst + 1, dst + 1, base_s + 1)))
    E(Op("s_branch", (f".Lsgd{tag}",)))
    E(Op("label", (f".Lsgs{tag}",)))
    E(Op("s_mul", (dst, g, gs_s)))
    E(Op("s_mul_hi", (dst + 1, g, gs_s)))
    E(Op("s_add_cc", (dst, dst, base_s)))
    E(Op("s_addc", (dst + 1, dst + 1, base_s + 1)))
    E(Op("label", (f".Lsgd{tag}",)))


SW_SKIP = 81   # xchg synw: 1 when the item's generations accepted no repair of this pass


def _synw_item_setup(E, spec: KernelSpec):
    """Per item: g0 / g1, the four load-lane masks, both generations' row
    bases and slot-map pointers; items whose generations accepted no repair
    of this pass (bound <= j0 for both) skip to the next item (xchg: set
    s[SW_SKIP] instead -- the wave still produces its share of the rows)."""
    E(Op("s_exec", (None,)))
    E(Op("v_readfirstlane", (SW_G0, V_GA)))          # lane 0, unit A: the item's first unit
    E(Op("s_addk", (SW_G1, SW_G0, 1)))
    E(Op("s_min", (SW_G1, SW_G1, SW_GLAST)))
    for gv, vm, m0, m1 in ((V_GA, 26, SW_A0, SW_A1), (V_GB, 24, SW_B0, SW_B1)):
        E(Op("v_cmp_eq_s", (S_TMP, SW_G0, gv)))
        E(Op("s_nop", (4,)))
        E(Op("s_and64", (m0, vm, S_TMP)))
        E(Op("s_andn2_64", (m1, vm, S_TMP)))
    for t, (g, R, Mp) in enumerate(((SW_G0, SW_R0, SW_M0), (SW_G1, SW_R1, SW_M1))):
        _scalar_gen_base(E, R, 4, 8, S_OFFS, g, f"r{t}")
        E(Op("s_mul", (Mp, g, 19)))
        E(Op("s_mul_hi", (Mp + 1, g, 19)))
        E(Op("s_add_cc", (Mp, Mp, 20)))
        E(Op("s_addc", (Mp + 1, Mp + 1, 21)))
    # pass skip: no lane's generation accepted a repair >= j0
    E(Op("s_cmp_eq64_0_br", (SW_BOUND, ".Lnobound")))
    for t, g in enumerate((SW_G0, SW_G1)):
        E(Op("s_lshl", (SW_BASE0, g, 2)))
        E(Op("s_add_cc", (SW_BASE0, SW_BASE0, SW_BOUND)))
        E(Op("s_addck", (SW_BASE0 + 1, SW_BOUND + 1, 0)))
        E(Op("s_load_x1", (SW_T0 + t, SW_BASE0, 0)))
        E(Op("s_waitcnt_lgkm", ()))
    E(Op("s_max", (SW_T0, SW_T0, SW_T1)))
    E(Op("s_cmp_le_k_br", (SW_T0, spec.j0, ".Lskipnear")))
    E(Op("s_branch", (".Lnobound",)))
    E(Op("label", (".Lskipnear",)))
    if spec.xchg:
        E(Op("s_movk", (SW_SKIP, 1)))
        E(Op("s_branch", (".Lsetup_end",)))
    else:
        E(Op("s_far_jump", (".Lskip", 2)) if spec.far else Op("s_branch", (".Lskip",)))
    E(Op("label", (".Lnobound",)))
    if spec.xchg:
        E(Op("s_movk", (SW_SKIP, 0)))
        E(Op("label", (".Lsetup_end",)))


def _synw_load_row(E, spec: KernelSpec, quad: list, kind: str, idx: int, b: int):
    """Loads of source row idx ("src") or pass repair idx ("rep") of both of
    the item's generations into b .. b + 7 (the zero row where the slot map
    says absent): the slot byte from the scalar map quad (re-read when the
    row's quad changes, quad[0] tracks it), four masked saddr loads."""
    k = spec.k
    pos = k + spec.j0 + idx if kind == "rep" else idx
    q = pos // 16
    if quad[0] != q:
        E(Op("s_load_x4", (SW_Q0, SW_M0, 16 * q)))
        E(Op("s_load_x4", (SW_Q1, SW_M1, 16 * q)))
        E(Op("s_waitcnt_lgkm", ()))
        quad[0] = q
    w, sh = (pos % 16) // 4, 8 * (pos % 4)
    for qb, base, R, t in ((SW_Q0, SW_BASE0, SW_R0, SW_T0), (SW_Q1, SW_BASE1, SW_R1, SW_T1)):
        E(Op("s_bfe_k", (t, qb + w, sh, 8)))
        E(Op("s_mul", (base, t, 10)))
        E(Op("s_mul_hi", (base + 1, t, 10)))
        E(Op("s_add_cc", (base, base, R)))
        E(Op("s_addc", (base + 1, base + 1, R + 1)))
        E(Op("s_cmp_eq_k", (t, ABSENT)))
        E(Op("s_cselect64", (base, 22, base)))
    for mask, voff, d, sb in ((SW_A0, V_SRCA, b, SW_BASE0), (SW_A1, V_SRCA, b, SW_BASE1),
                              (SW_B0, V_SRCB, b + 4, SW_BASE0), (SW_B1, V_SRCB, b + 4, SW_BASE1)):
        E(Op("s_exec", (mask,)))
        if not spec.lab_norows:
            E(Op("load16_saddr", (d, voff, sb, spec.ld_policy)))
    E(Op("s_exec", (None,)))


def _generate_synw(spec: KernelSpec) -> list[Op]:
    """Decode stage A for long rows (padded units per row >= 128): syndromes
    s_j = p_j ^ sum_{i present} C[j][i] x_i of repairs j0 .. j0 + r - 1 of the
    (k, r_total) code, for every unit of every generation, without the slot
    map in VGPRs -- so it takes r up to 22 per pass at any k.

    An item (128 consecutive units) lies in at most two generations.  For
    each row the scalar unit loads the slot bytes of both (one 16-byte map
    quad per 16 rows and generation), forms the row address of each (the
    zero row when absent) and the halves load with it as saddr plus 16 u,
    under the lanes of the respective generation (four loads per row).
    Rows stream as in _generate_syn (repairs initialise the accumulators);
    syndromes of all r repairs are stored, the unaccepted ones are junk the
    combine never reads."""
    if spec.xchg:
        return _generate_xchg(spec)
    k, r, pd, nbuf = spec.k, spec.r, spec.pd, spec.nbuf
    C = cauchy(k, spec.rt)[spec.j0: spec.j0 + r]
    acc0, ring0 = spec.acc0, spec.ring0
    seq = [("rep", j) for j in range(r)] + [("src", i) for i in range(k)]
    ops: list[Op] = []
    E = ops.append
    _prologue(E, spec)
    _synw_item_setup(E, spec)
    quad = [None]

    def load_row(n: int, b: Optional[int] = None, order=seq):
        if b is None:
            b = ring0 + 8 * (n % nbuf)
        _synw_load_row(E, spec, quad, *order[n], b)

    n_seq = len(seq)
    per_row = 0 if spec.lab_norows else 4
    if spec.fft:
        # additive-FFT syndromes (lch_fft plan of the pass, as the 'N' encode):
        # sources (the zero row when absent) through the chunked transform,
        # then each repair row, in byte form, onto its transposed block
        P = spec.fplan
        fseq = [("src", i) for i in P.order] + [("rep", j) for j in range(r)]
        n_all = len(fseq)

        def load_fft(n: int, base: int):
            load_row(n, base, fseq)

        def wait_fft(n: int):
            E(Op("s_waitcnt_vm", (per_row * min(pd, n_all - 1 - n),)))

        _fft_stream(E, ops, spec, load_fft, wait_fft, lambda t: acc0 + 8 * t, n_rows=n_all)
        for n in range(k, n_all):
            if n + pd < n_all:
                load_fft(n + pd, ring0 + 8 * ((n + pd) % nbuf))
            wait_fft(n)
            blk0 = acc0 + 8 * P.out_block[fseq[n][1]]
            ops.extend(_transpose_ops(blk0, spec.bfi_transpose, spec.vmask))
            base = ring0 + 8 * (n % nbuf)
            for b in range(8):
                E(Op("v_xor", (blk0 + b, blk0 + b, base + b)))
        E(Op("s_nop", (4,)))
        for j in range(r):
            _store_pair(E, acc0 + 8 * P.out_block[j], S_STA, S_STB, spec.st_policy)
        E(Op("label", (".Lskip",)))
        _epilogue_next_item(E, far=spec.far)
        return ops
    for n in range(min(pd, n_seq)):
        load_row(n)
    for n, (kind, idx) in enumerate(seq):
        if n + pd < n_seq:
            load_row(n + pd)
        after = min(pd, n_seq - 1 - n)
        E(Op("s_waitcnt_vm", (per_row * after,)))
        base = ring0 + 8 * (n % nbuf)
        if kind == "rep":
            ops.extend(_transpose_ops(base, spec.bfi_transpose, spec.vmask))
            for b in range(8):
                E(Op("v_mov", (acc0 + 8 * idx + b, base + b)))
        else:
            _source_row(ops, C, idx, r, base, acc0, init=False, xor3=spec.xor3, bfi=spec.bfi_transpose, vmask=spec.vmask)
    for j in range(r):
        ops.extend(_transpose_ops(acc0 + 8 * j, spec.bfi_transpose, spec.vmask))
    E(Op("s_nop", (4,)))
    for j in range(r):
        _store_pair(E, acc0 + 8 * j, S_STA, S_STB, spec.st_policy)
    E(Op("label", (".Lskip",)))
    _epilogue_next_item(E, far=spec.far)
    return ops


# --------------------------------------------------------------------------
# Fused decode, lane-chunk layout (spec.chunked)
# --------------------------------------------------------------------------
S_QB = 76   # s[76:77] = {16 Q, 0}: byte offset of a lane's B unit from its A unit
S_TAIL = 78  # s[78:79]: the lane whose B unit is the partial last unit (L % 16 = s59 != 0)


def lu_layout_chunked(spec) -> dict:
    """LU-phase registers of the chunked dec kernel (all dead in the row loop
    unless noted): 16 column quads over the ring, the slot map and the top of
    the file; the rank quad in the B-pointer / spare pointer registers."""
    sel = 18                                 # 24 selectors: v18..v41 (combos, zero pointers)
    if spec.fft:
        # additive-FFT layout: the ring (pd + ch slots, dead in the LU phase)
        # holds the r column quads, then the table buffers and record pointer
        # (lds_rows: the ring is only the chunk; those go above the accumulators)
        cols = [spec.ring0 + 4 * q for q in range(spec.r)]
        top = spec.ring0 + 4 * spec.r
        if spec.lds_rows:
            top = spec.acc0 + 8 * spec.nacc
            assert 4 * spec.r <= 8 * spec.nbuf
        tb = (top, top + 6)
        ta = (top + 5, top + 11)
        fp = top + 12
        end = fp + 2
        assert spec.lds_rows or end <= spec.ring0 + 8 * spec.nbuf, "LU registers exceed the ring"
        if spec.lu_ahead == 2:
            # three buffers (b128 base, b32 register): the third one's b128 over
            # the record pointer (dead once the record loads are issued) and the
            # next pair, its b32 in the second address register; one address
            # register for all (a read takes its address at issue)
            assert not spec.lds_rows and top % 2 == 0
            tbx = ((top, top + 4), (top + 6, top + 10), (top + 12, top + 11))
            end = top + 16
            assert end <= spec.ring0 + 8 * spec.nbuf, "LU registers exceed the ring"
            return {"cols": cols, "rank": V_SRCA, "sel": sel, "tb": tb, "ta": (top + 5,) * 3, "fp": fp,
                    "end": end, "tbx": tbx}
        return {"cols": cols, "rank": V_SRCA, "sel": sel, "tb": tb, "ta": ta, "fp": fp, "end": end,
                "tbx": ((tb[0], tb[0] + 4), (tb[1], tb[1] + 4))}
    cols = [spec.ring0 + 4 * q for q in range(2 * spec.nbuf)]
    cols += [spec.map_a + 4 * q for q in range(spec.map_quads)]
    top = spec.map_a + 4 * spec.map_quads
    top = (top + 3) // 4 * 4
    tb = (top, top + 6)                      # two table buffers of 5 dwords (b128 at even registers)
    ta = (top + 5, top + 11)
    fp = top + 12                            # LU record pointer (2)
    nxt = top + 14
    nxt = (nxt + 3) // 4 * 4
    while len(cols) < spec.r:
        cols.append(nxt)
        nxt += 4
    if not spec.lu and not spec.lab_lu_only:   # lab: stores only (record pointer in the dead ring)
        return {"cols": cols[: spec.r], "rank": V_SRCA, "sel": sel, "tb": tb, "ta": ta, "fp": spec.ring0,
                "end": top}
    return {"cols": cols[: spec.r], "rank": V_SRCA, "sel": sel, "tb": tb, "ta": ta, "fp": fp,
            "end": max(nxt, fp + 2)}


def _prologue_chunked(E, spec: KernelSpec):
    """Prologue of the chunked dec kernel: lane-chunk f = 64 item + lane,
    g = f / Q, q = f % Q; A unit q, B unit q + Q (loaded iff q + Q < Lu).
    kernarg s12 = Lu, s13 = Q, s14 = G * Q, s15 / s16 = magic / shift of Q."""
    if spec.lab_stamps:
        E(Op("stamp", (0,)))
    E(Op("s_load_args", ()))
    E(Op("v_lshr", (V_T, 6, V_LANE)))
    E(Op("v_andk", (V_LANE, 63, V_LANE)))
    E(Op("v_readfirstlane", (29, V_T)))
    E(Op("s_load_args_dec", ()))
    E(Op("s_load_args_offs", (spec.offs_kernarg,)))
    if spec.mode == "synw":
        E(Op("s_load_karg_x2", (SW_BOUND, KERNARG_BYTES)))   # kernarg words 24..25
    E(Op("s_nop", (4,)))
    E(Op("s_waitcnt_lgkm", ()))
    # split tables -> LDS (as _prologue; the closed-form solve has no tables)
    ts = spec.tab_stride
    if not spec.cx:
        E(Op("s_movk", (62, 4096)))
        E(Op("s_movk", (63, 0)))
        E(Op("v_movs", (V_ADDR, 60)))
        E(Op("v_movs", (V_ADDR + 1, 61)))
        E(Op("v_mad64_k", (V_ADDR, V_LANE, 16, V_ADDR)))
        E(Op("v_add64_s", (V_SRCA, V_ADDR, 62)))
        for q in range(8):
            E(Op("load16", (48 + 4 * q, V_ADDR if q < 4 else V_SRCA, 1024 * (q % 4))))
        # global bytes q*1024 + 16 l = record 32 q + l/2, half l % 2 -> LDS
        # (32 q + l/2) * stride + 16 (l % 2)
        E(Op("v_lshr", (V_T, 1, V_LANE)))
        E(Op("v_lshl", (V_T, ts.bit_length() - 1, V_T)))
        E(Op("v_andk", (V_T + 1, 1, V_LANE)))
        E(Op("v_lshl", (V_T + 1, 4, V_T + 1)))
        E(Op("v_xor", (V_T, V_T, V_T + 1)))
        for b in range(4):
            E(Op("s_movk", (S_PICK + b, 0x0C0C000C | (b << 8))))
        E(Op("s_waitcnt_vm", (0,)))
        for q in range(8):
            E(Op("ds_write_b128", (V_T, 48 + 4 * q, 32 * ts * q)))
        E(Op("s_waitcnt_lgkm_n", (0,)))
    if spec.lds_rows:   # this wave's row slots: after the tables, lds_rows x 2 KiB per wave
        E(Op("s_movk", (S_ROWLDS, spec.lds_rows * LDS_ROW_BYTES)))
        E(Op("s_mul", (S_ROWLDS, S_ROWLDS, 29)))
        if not spec.cx:   # after the split tables (the closed-form solve has none)
            E(Op("s_addk", (S_ROWLDS, S_ROWLDS, 256 * ts)))
        E(Op("v_lshl", (V_LDSA, 4, V_LANE)))
        E(Op("v_add_s", (V_LDSA, S_ROWLDS, V_LDSA)))
    if spec.xcd_remap:
        E(Op("s_lshrk", (46, 18, 2)))
        E(Op("s_andk", (47, 2, 7)))
        E(Op("s_lshrk", (30, 46, 3)))
        E(Op("s_mul", (30, 47, 30)))
        E(Op("s_andk", (46, 46, 7)))
        E(Op("s_min", (46, 47, 46)))
        E(Op("s_add", (30, 30, 46)))
        E(Op("s_lshrk", (46, 2, 3)))
        E(Op("s_add", (30, 30, 46)))
        E(Op("s_lshl", (30, 30, 2)))
    else:
        E(Op("s_lshl", (30, 2, 2)))
    if spec.ksplit > 1:
        E(Op("s_lshrk", (28, 30, 2)))          # the workgroup's item (all its waves)
    else:
        E(Op("s_add", (28, 29, 30)))
    E(Op("s_mov", (32, 10)))
    E(Op("s_movk", (33, 0)))
    E(Op("s_mov", (34, 11)))
    E(Op("s_movk", (35, 0)))
    E(Op("s_lshl", (S_QB, 13, 4)))           # 16 Q
    E(Op("s_movk", (S_QB + 1, 0)))
    E(Op("s_movk", (S_ABSENT, ABSENT)))
    if spec.mode == "synw":   # G - 1 = (total - 1) / Lv
        E(Op("s_addk", (SW_GLAST, 14, -1)))
        E(Op("s_mul_hi", (SW_GLAST, SW_GLAST, 15)))
        E(Op("s_lshr_s", (SW_GLAST, SW_GLAST, 16)))
    for q, (_, mask, _) in enumerate(_TRANSPOSE):
        E(Op("s_movk", (S_TMASK + q, mask)))
    if spec.vmask is not None:
        for q in range(3):
            E(Op("v_movs", (spec.vmask[q], S_TMASK + q)))
    E(Op("label", (".Litem",)))
    E(Op("s_cmp_lt_br", (28, 17, ".Lgo")))
    E(Op("s_far_jump", (".Lend", 0)))
    E(Op("label", (".Lgo",)))
    if spec.lab_stamps:
        E(Op("stamp", (1,)))
    if spec.wave_gen:
        # f = Q item + (lane < Q ? lane : 0): lanes past Q alias lane 0 and store nothing
        E(Op("v_cmp_gt_s", (26, 13, V_LANE)))
        E(Op("v_movk", (V_T, 0)))
        E(Op("s_nop", (4,)))
        E(Op("v_cndmask", (V_T, V_T, V_LANE, 26)))
        E(Op("s_mul", (S_TMP, 28, 13)))
        E(Op("v_add_s", (V_F, S_TMP, V_T)))
    else:
        E(Op("v_lshl_add_s", (V_F, 28, 6, V_LANE)))   # f = 64 item + lane
        E(Op("v_cmp_gt_s", (26, 14, V_F)))             # f < G * Q
    E(Op("v_mul_hi_s", (V_GA, V_F, 15)))
    E(Op("v_lshr_s", (V_GA, 16, V_GA)))            # g
    E(Op("v_mul_lo_s", (V_UA, V_GA, 13)))
    E(Op("v_sub", (V_UA, V_F, V_UA)))              # q
    E(Op("v_add_s", (V_UB, 13, V_UA)))             # q + Q
    E(Op("v_cmp_gt_s", (S_PAD, 12, V_UB)))         # q + Q < Lu
    E(Op("s_nop", (4,)))
    E(Op("s_and64", (S_TMP2, 26, 26)))
    E(Op("s_and64", (24, 26, S_PAD)))
    E(Op("s_and64", (S_STA, 26, 26)))
    E(Op("s_and64", (S_STB, 24, 24)))
    if spec.mode == "dec" and spec.chunked:
        # L % 16 != 0 (s59 = kernarg word 23): the last unit Lu - 1 is some
        # lane's unit B; that lane stores it bytewise, the others whole
        E(Op("s_movk", (S_TAIL, 0)))
        E(Op("s_movk", (S_TAIL + 1, 0)))
        E(Op("s_cmp_eq_k_br", (59, 0, ".Lnotail")))
        E(Op("s_addk", (S_TMP, 12, -1)))
        E(Op("v_cmp_eq_s", (S_TAIL, S_TMP, V_UB)))
        E(Op("s_nop", (4,)))
        E(Op("s_and64", (S_TAIL, S_TAIL, S_STB)))
        E(Op("s_andn2_64", (S_STB, S_STB, S_TAIL)))
        E(Op("label", (".Lnotail",)))
    _gen_base(E, V_SRCA, 4, 8, S_OFFS, V_GA, S_TMP2, "r")
    E(Op("v_mad64_k", (V_SRCA, V_UA, 16, V_SRCA)))
    _gen_base(E, V_DSTA, 6, 9, S_OFFS + 2, V_GA, S_TMP2, "d")
    E(Op("v_mad64_k", (V_DSTA, V_UA, 16, V_DSTA)))
    E(Op("v_movs", (V_ZA, 22)))
    E(Op("v_movs", (V_ZA + 1, 23)))
    E(Op("v_mad64_k", (V_ZA, V_UA, 16, V_ZA)))
    if spec.lab_zspread:
        E(Op("v_andk", (V_SLOT, 63, V_GA)))
        E(Op("v_lshl", (V_SLOT, 11, V_SLOT)))
        E(Op("v_mad64_k", (V_ZA, V_SLOT, 1, V_ZA)))
    E(Op("s_nop", (4,)))
    E(Op("label", (".Lbody",)))


def _generate_dec_chunked(spec: KernelSpec) -> list[Op]:
    """Fused decode (syndromes + in-register LU solve, as _generate_syn's dec
    mode) over the lane-chunk layout: each lane's 32 bytes belong to one
    generation, so the slot-map gather runs once per row (B address = A +
    16 Q), and the LU reads each coefficient's split tables once for all 8
    dwords of a block."""
    k, r, pd, nbuf = spec.k, spec.r, spec.pd, spec.nbuf
    C = cauchy(k, r)
    acc0, ring0, mp = spec.acc0, spec.ring0, spec.map_a
    ops: list[Op] = []
    E = ops.append
    _prologue_chunked(E, spec)
    # the generation's slot map (payload lanes; padding-free: every lane with a chunk)
    # (additive FFT with more than FFT_MAP_DEC_QUADS map quads, k + r > 80: a
    # window of FFT_MAP_DEC_QUADS quads in v18..; the quads past it sit in the
    # free ring for the jmax scan, and once the row loop reaches them they are
    # reloaded over the window's first quads, whose rows have all been issued)
    W = FFT_MAP_DEC_QUADS if spec.fft and spec.map_quads > FFT_MAP_DEC_QUADS else spec.map_quads
    win = {"phase": 0}

    def map_load(quads, reg):
        E(Op("v_movs", (V_ADDR, 20)))
        E(Op("v_movs", (V_ADDR + 1, 21)))
        E(Op("v_mad64_s", (V_ADDR, V_GA, 19, V_ADDR)))
        E(Op("s_exec", (S_STA,)))
        for q in quads:
            E(Op("load16", (reg(q), V_ADDR, 16 * q)))
        E(Op("s_exec", (None,)))
        E(Op("s_waitcnt_vm", (0,)))
    map_load(range(spec.map_quads), lambda q: mp + 4 * q if q < W else ring0 + 4 * (q - W))
    seq = [("src", i) for i in range(k)] + [("rep", j) for j in range(r)]

    def map_reg(pos: int) -> int:
        q = pos // 16
        if q < W:
            assert win["phase"] < 2, "map quad reloaded over"
            return mp + pos // 4
        if win["phase"] == 0:
            return ring0 + 4 * (q - W) + (pos % 16) // 4
        if win["phase"] == 1:    # the row loop reaches the quads past the window
            map_load(range(W, spec.map_quads), lambda qq: mp + 4 * (qq - W))
            win["phase"] = 2
        return mp + 4 * (q - W) + (pos % 16) // 4

    def present(pos: int, sm: int):
        E(Op("v_bfe", (V_SLOT, map_reg(pos), 8 * (pos % 4), 8)))
        E(Op("v_cmp_ne_s", (sm, S_ABSENT, V_SLOT)))
        E(Op("s_nop", (4,)))

    # jmax over the item's payload lanes
    for j in reversed(range(r)):
        present(k + j, S_TMP)
        E(Op("s_and64", (S_TMP, S_TMP, S_STA)))
        E(Op("s_movk", (S_JMAX, j + 1)))
        E(Op("s_cmp_lg64_br", (S_TMP, ".Ljdone")))
    E(Op("s_movk", (S_JMAX, 0)))
    E(Op("label", (".Ljdone",)))
    win["phase"] = 1
    if spec.lab_stamps:
        E(Op("stamp", (2,)))
    if spec.wave_gen:   # any source row may be skipped, so no row initialises
        for a in range(acc0, acc0 + 8 * r):
            E(Op("v_movk", (a, 0)))

    def load_row(n: int, slot: Optional[int] = None):
        b = ring0 + 8 * ((n if slot is None else slot) % nbuf)
        kind, idx = seq[n]
        present(idx if kind == "src" else k + idx, S_TMP)
        E(Op("v_mad64_s", (V_ADDR, V_SLOT, 10, V_SRCA)))
        E(Op("v_cndmask", (V_ADDR, V_ZA, V_ADDR, S_TMP)))
        E(Op("v_cndmask", (V_ADDR + 1, V_ZA + 1, V_ADDR + 1, S_TMP)))
        E(Op("v_add64_s", (V_SRCB, V_ADDR, S_QB)))
        E(Op("s_exec", (26,)))
        if not spec.lab_norows:
            E(Op("load16", (b, V_ADDR, 0, spec.ld_policy)))
        E(Op("s_exec", (24,)))
        if not spec.lab_norows:
            E(Op("load16", (b + 4, V_SRCB, 0, spec.ld_policy)))
        E(Op("s_exec", (None,)))

    n_seq = 0 if spec.lab_lu_only else len(seq)
    if spec.ksplit > 1:
        _dec_ksplit(E, ops, spec, seq, load_row, present)
        return ops
    if spec.fft:
        assert not (spec.wave_gen or spec.lab_lu_only)
        P = spec.fplan
        fseq = [("src", i) for i in P.order] + [("rep", j) for j in range(r)]
        n_all = len(fseq)

        S = spec.lds_rows
        ahead = spec.ahead

        def load_fft(n: int, base: int):
            kind, idx = fseq[n]
            if spec.lab_slot_order:
                E(Op("v_movk", (V_SLOT, n % 64)))
            else:
                present(idx if kind == "src" else k + idx, S_TMP)
            E(Op("v_mad64_s", (V_ADDR, V_SLOT, 10, V_SRCA)))
            if not (spec.lab_slot_order or spec.lab_skip_absent):
                E(Op("v_cndmask", (V_ADDR, V_ZA, V_ADDR, S_TMP)))
                E(Op("v_cndmask", (V_ADDR + 1, V_ZA + 1, V_ADDR + 1, S_TMP)))
            E(Op("v_add64_s", (V_SRCB, V_ADDR, S_QB)))
            for h, (vm, va) in enumerate(((26, V_ADDR), (24, V_SRCB))):
                if spec.lab_skip_absent and not spec.lab_slot_order:
                    E(Op("s_and64", (S_TMP2, vm, S_TMP)))
                    E(Op("s_exec", (S_TMP2,)))
                else:
                    E(Op("s_exec", (vm,)))
                if spec.lab_norows:
                    continue
                if S:   # -> LDS slot n % S of this wave (no VGPR destination)
                    E(Op("s_m0", (S_ROWLDS, (n % S) * LDS_ROW_BYTES + 1024 * h)))
                    E(Op("load16_lds", (va, spec.ld_policy)))
                else:
                    E(Op("load16", (base + 4 * h, va, 0, spec.ld_policy)))
            E(Op("s_exec", (None,)))

        def wait_fft(n: int):
            E(Op("s_waitcnt_vm", (0 if spec.lab_norows else 2 * min(ahead, n_all - 1 - n),)))
            if S:   # the row from its LDS slot into the chunk registers
                base = ring0 + 8 * (n % nbuf)
                E(Op("ds_read_b128", (base, V_LDSA, (n % S) * LDS_ROW_BYTES)))
                E(Op("ds_read_b128", (base + 4, V_LDSA, (n % S) * LDS_ROW_BYTES + 1024)))
                E(Op("s_waitcnt_lgkm_n", (0,)))

        if spec.prio != (0, 0):
            E(Op("s_setprio", (spec.prio[0],)))
        if spec.cx:
            # repair rows rotate through three ring slots (the first two are
            # where _fft_stream loaded rows k and k + 1), away from slots 8
            # and 9, which take the record's alpha quads (_cx_solve)
            rot = cx_repair_slots(spec)

            def cx_slot(n):
                if spec.lds_rows and n >= k:
                    return ring0 + 8 * rot[(n - k) % 3]
                return ring0 + 8 * (n % nbuf if n < k else rot[(n - k) % 3])
            _fft_stream(E, ops, spec, load_fft, wait_fft, lambda t: acc0 + 8 * t, n_rows=n_all)
            if spec.lab_stamps:
                E(Op("stamp", (3,)))
            _cx_solve(E, ops, spec, P, fseq, load_fft, cx_slot)
            if spec.lab_stamps:
                E(Op("stamp", (6,)))
                E(Op("stamp_flush", ()))
            _epilogue_next_item(E, far=True)
            return ops
        _fft_stream(E, ops, spec, load_fft, wait_fft, lambda t: acc0 + 8 * t, n_rows=n_all)
        if spec.lab_stamps:
            E(Op("stamp", (3,)))
        # the accepted repairs, in byte form, onto their syndrome blocks
        for n in range(k, n_all):
            if n + ahead < n_all:
                load_fft(n + ahead, ring0 + 8 * ((n + ahead) % nbuf))
            wait_fft(n)
            j = fseq[n][1]
            blk0 = acc0 + 8 * P.out_block[j]
            E(Op("s_cmp_le_k_br", (S_JMAX, j, f".Lrep{j}")))
            ops.extend(_transpose_ops(blk0, spec.bfi_transpose, spec.vmask))
            base = ring0 + 8 * (n % nbuf)
            for b in range(8):
                E(Op("v_xor", (blk0 + b, blk0 + b, base + b)))
            E(Op("label", (f".Lrep{j}",)))
        if spec.prio != (0, 0):
            E(Op("s_setprio", (spec.prio[1],)))
        if spec.lab_stamps:
            E(Op("stamp", (4,)))
        _lu_solve_and_store_chunked(E, spec)
        if spec.lab_stamps:
            E(Op("stamp", (6,)))
            E(Op("stamp_flush", ()))
        _epilogue_next_item(E, far=True)
        return ops
    for n in range(min(pd, n_seq)):
        load_row(n)
    for n, (kind, idx) in enumerate(seq[:n_seq]):
        if n + pd < n_seq:
            load_row(n + pd)
        after = min(pd, n_seq - 1 - n)
        E(Op("s_waitcnt_vm", (0 if spec.lab_norows else 2 * after,)))
        base = ring0 + 8 * (n % nbuf)
        if kind == "rep":
            E(Op("s_cmp_le_k_br", (S_JMAX, idx, f".Lrep{idx}")))
            ops.extend(_transpose_ops(acc0 + 8 * idx, spec.bfi_transpose, spec.vmask))
            for b in range(8):
                E(Op("v_xor", (acc0 + 8 * idx + b, acc0 + 8 * idx + b, base + b)))
            E(Op("label", (f".Lrep{idx}",)))
        elif spec.wave_gen:
            present(idx, S_TMP)
            E(Op("s_and64", (S_TMP, S_TMP, S_STA)))
            E(Op("s_cmp_eq64_0_br", (S_TMP, f".Lskip{n}")))
            _source_row(ops, C, idx, r, base, acc0, init=False, xor3=spec.xor3, bfi=spec.bfi_transpose, vmask=spec.vmask,
                        guard=(spec.guard_min, f".Lrow{n}"))
            E(Op("label", (f".Lskip{n}",)))
        else:
            _source_row(ops, C, idx, r, base, acc0, init=idx == 0, xor3=spec.xor3, bfi=spec.bfi_transpose, vmask=spec.vmask,
                        guard=(spec.guard_min, f".Lrow{n}"))
    _lu_solve_and_store_chunked(E, spec)
    _epilogue_next_item(E, far=True)
    return ops


# lu_ilp: product temps of up to three interleaved dwords -- R_P and low VGPRs
# the chunked kernel uses only in its row loop or stores (v17, v43, V_ADDR,
# V_SLOT, v47), free during the LU whatever the (k, r) layout above v48
LU_ILP_TEMPS = (R_P, R_P + 1, R_P + 2, 17, 43, V_ADDR, V_ADDR + 1, V_SLOT, 47)
LU_ILP_GROUPS = ((0, 1, 2), (3, 4, 5), (6, 7))


def _prefetch_setup(E, spec: KernelSpec):
    """lab_prefetch: v[44:45] <- the next item's row-0 address of each lane
    (strided generations), s[38:39] / s[40:41] the lanes whose A / B unit
    exists; no next item -> skip to .Lnopf."""
    E(Op("s_add", (46, 28, 18)))
    E(Op("s_cmp_ge_br", (46, 17, ".Lnopf_far")))
    E(Op("v_lshl_add_s", (14, 46, 6, V_LANE)))
    E(Op("v_cmp_gt_s", (S_TMP, 14, 14)))              # f' < G Q
    E(Op("v_mul_hi_s", (15, 14, 15)))
    E(Op("v_lshr_s", (15, 16, 15)))                   # g'
    E(Op("v_mul_lo_s", (16, 15, 13)))
    E(Op("v_sub", (16, 14, 16)))                      # q'
    E(Op("v_add_s", (17, 13, 16)))
    E(Op("v_cmp_gt_s", (S_TMP2, 12, 17)))             # q' + Q < Lu
    E(Op("s_nop", (4,)))
    E(Op("s_and64", (S_TMP2, S_TMP2, S_TMP)))
    E(Op("v_movs", (V_ADDR, 4)))
    E(Op("v_movs", (V_ADDR + 1, 5)))
    E(Op("v_mad64_s", (V_ADDR, 15, 8, V_ADDR)))
    E(Op("v_mad64_k", (V_ADDR, 16, 16, V_ADDR)))
    E(Op("s_branch", (".Lpf_go",)))
    E(Op("label", (".Lnopf_far",)))
    E(Op("s_exec", (None,)))
    E(Op("s_movk", (S_TMP, 0)))                       # no next item: empty load masks
    E(Op("s_movk", (S_TMP + 1, 0)))
    E(Op("s_movk", (S_TMP2, 0)))
    E(Op("s_movk", (S_TMP2 + 1, 0)))
    E(Op("label", (".Lpf_go",)))


def _prefetch_rows(E, spec: KernelSpec, n: int):
    _, boff = spec.lab_prefetch
    for _ in range(n):
        E(Op("s_exec", (S_TMP,)))
        E(Op("load4", (47, V_ADDR, 0)))
        E(Op("s_exec", (S_TMP2,)))
        E(Op("load4", (47, V_ADDR, boff)))
        E(Op("s_exec", (None,)))
        E(Op("v_add64_s", (V_ADDR, V_ADDR, 32)))      # + row stride


def _dec_ksplit(E, ops: list, spec: KernelSpec, seq, load_row, present):
    """ksplit body of the chunked fused decode: wave w of the workgroup runs
    rows w, w + ks, w + 2 ks, ... of the item (same slot map, same lanes),
    leaves every block < jmax in byte form (a block's transpose is linear, so
    partial sums transpose like the whole), waves 1.. write their blocks to
    LDS, wave 0 adds them in, solves and stores while the others start the
    next item.  Two barriers per item: partials written / partials read."""
    k, r, pd, nbuf, ks = spec.k, spec.r, spec.pd, spec.nbuf, spec.ksplit
    C = cauchy(k, r)
    acc0, ring0 = spec.acc0, spec.ring0
    for w in range(1, ks):
        E(Op("s_cmp_lg_k_br", (29, w, f".Lnsec{w}")))
        E(Op("s_far_jump", (f".Lsec{w}", 40 + w)))
        E(Op("label", (f".Lnsec{w}",)))
    for w in range(ks):
        E(Op("label", (f".Lsec{w}",)))
        rows = [n for n in range(len(seq)) if n % ks == w]
        srcs = [seq[n][1] for n in rows if seq[n][0] == "src"]
        owned = {seq[n][1] for n in rows if seq[n][0] == "rep"}
        if not srcs:   # no source row initialises the accumulators
            for a in range(acc0, acc0 + 8 * r):
                E(Op("v_movk", (a, 0)))
        for m in range(min(pd, len(rows))):
            load_row(rows[m], m)
        for m, n in enumerate(rows):
            if m + pd < len(rows):
                load_row(rows[m + pd], m + pd)
            after = min(pd, len(rows) - 1 - m)
            E(Op("s_waitcnt_vm", (2 * after,)))
            base = ring0 + 8 * (m % nbuf)
            kind, idx = seq[n]
            if kind == "rep":
                E(Op("s_cmp_le_k_br", (S_JMAX, idx, f".Lrep{idx}")))
                ops.extend(_transpose_ops(acc0 + 8 * idx, spec.bfi_transpose, spec.vmask))
                for b in range(8):
                    E(Op("v_xor", (acc0 + 8 * idx + b, acc0 + 8 * idx + b, base + b)))
                E(Op("label", (f".Lrep{idx}",)))
            else:
                _source_row(ops, C, idx, r, base, acc0, init=idx == srcs[0], xor3=spec.xor3,
                            bfi=spec.bfi_transpose, vmask=spec.vmask, guard=(spec.guard_min, f".Lrow{n}"))
        # blocks whose repair row another wave holds: back to byte form here
        for j in range(r):
            if j in owned:
                continue
            E(Op("s_cmp_le_k_br", (S_JMAX, j, f".Lbt{w}_{j}")))
            ops.extend(_transpose_ops(acc0 + 8 * j, spec.bfi_transpose, spec.vmask))
            E(Op("label", (f".Lbt{w}_{j}",)))
        if w + 1 < ks:
            E(Op("s_far_jump", (".Lsec_end", 50 + w)))
    E(Op("label", (".Lsec_end",)))
    _ksplit_reduce(E, ks, r, acc0, V_ADDR, ring0, LDS_TAB_BYTES, jmax_guard=True)
    _lu_solve_and_store_chunked(E, spec)
    _ksplit_epilogue(E)


def _ksplit_reduce(E, ks: int, nblk: int, acc0: int, areg: int, tmp: int, lds0: int, jmax_guard: bool):
    """Partial accumulator blocks (byte form) of waves 1..ks-1 -> LDS at
    lds0 + (w - 1) nblk 2 KiB, barrier, wave 0 XORs them into its own,
    barrier; waves 1.. then jump to .Lnext, wave 0 falls through.  areg and
    areg + 1: LDS address VGPRs, tmp..tmp+7: temps (dead registers)."""
    E(Op("v_lshl", (areg, 4, V_LANE)))              # LDS lane offset 16 l
    E(Op("s_cmp_eq_k_br", (29, 0, ".Lred0")))
    E(Op("s_addk", (46, 29, -1)))
    E(Op("s_movk", (47, nblk * KSPLIT_BLOCK_BYTES)))
    E(Op("s_mul", (46, 46, 47)))
    E(Op("s_addk", (46, 46, lds0)))
    E(Op("v_add_s", (areg, 46, areg)))
    for j in range(nblk):
        if jmax_guard:
            E(Op("s_cmp_le_k_br", (S_JMAX, j, ".Lwr_end")))
        E(Op("ds_write_b128", (areg, acc0 + 8 * j, KSPLIT_BLOCK_BYTES * j)))
        E(Op("ds_write_b128", (areg, acc0 + 8 * j + 4, KSPLIT_BLOCK_BYTES * j + 1024)))
    E(Op("label", (".Lwr_end",)))
    E(Op("s_waitcnt_lgkm_n", (0,)))
    E(Op("s_barrier", ()))
    E(Op("s_barrier", ()))
    E(Op("s_far_jump", (".Lnext", 60)))
    E(Op("label", (".Lred0",)))
    E(Op("s_barrier", ()))
    for w in range(1, ks):
        E(Op("v_addk", (areg + 1, lds0 + (w - 1) * nblk * KSPLIT_BLOCK_BYTES, areg)))
        for j in range(nblk):
            if jmax_guard:
                E(Op("s_cmp_le_k_br", (S_JMAX, j, f".Lrd_end{w}")))
            E(Op("ds_read_b128", (tmp, areg + 1, KSPLIT_BLOCK_BYTES * j)))
            E(Op("ds_read_b128", (tmp + 4, areg + 1, KSPLIT_BLOCK_BYTES * j + 1024)))
            E(Op("s_waitcnt_lgkm_n", (0,)))
            for b in range(8):
                E(Op("v_xor", (acc0 + 8 * j + b, acc0 + 8 * j + b, tmp + b)))
        E(Op("label", (f".Lrd_end{w}",)))
    E(Op("s_waitcnt_lgkm_n", (0,)))
    E(Op("s_barrier", ()))


def _ksplit_epilogue(E):
    E(Op("label", (".Lnext",)))
    E(Op("s_nop", (4,)))
    E(Op("s_lshrk", (46, 18, 2)))                     # item stride: the workgroups
    E(Op("s_add", (28, 28, 46)))
    E(Op("s_far_jump", (".Litem", 1)))
    E(Op("label", (".Lend",)))
    E(Op("s_endpgm", ()))


# --------------------------------------------------------------------------
# Closed-form Cauchy solve (spec.cx, round 6)
# --------------------------------------------------------------------------
# C[J,E]^-1 = diag(alpha) K diag(beta), K[b][a] = 1 / (x_a + y_b), x = k + J,
# y = E (lch_fft.cauchy_inverse_factors), and K is a sub-block of the fixed
# C^T: x_E = alpha * u|_E with u = C^T t, t_j = beta_j s_j (t_j = 0 for a
# repair the lane's generation did not accept).  u comes from the encode's
# additive-FFT plan run backwards with every op transposed
# (lch_fft.transposed_evaluate): the 16 syndrome blocks stay in registers and
# each chunk of 8 source rows is produced from them, then every row some lane
# of the wave recovers is scaled by its alpha, transposed back to bytes and
# stored.  The per-lane products are masked plane XORs (no v_perm, no LDS):
# c * y = XOR over the set bits a of c of y * 2^a, y * 2^a by in-place
# doubling (3 XORs a step, the planes renamed).
# Record (cx_record, CX_REC_BYTES): [0, 16) beta by repair index, [16, 24)
# the lane generation's erased-source mask, [32, 32 + k) alpha by source.
CX_REC_BYTES = 96
CX_MT = 38            # v38, v39: mask temps of the products
CX_ALPHA_SLOT = 8     # ring slots 8, 9: alpha (v112..v127)


def cx_regs(spec: KernelSpec) -> dict:
    """The cx solve's registers in the five slot-map quads v18..v37: beta,
    the erased mask, the product block `free` (two quads) and the store
    address pairs, around the quad holding the repair slots (k .. k + 15),
    which the repair loop still reads while the record lands."""
    repq = spec.k // 16
    q = [x for x in range(FFT_MAP_DEC_QUADS) if x != repq]
    beta, mask = q[0], q[1]
    rest = [x for x in range(FFT_MAP_DEC_QUADS) if x not in (beta, mask)]
    free = next(x for x in rest if x + 1 in rest)
    addr = next(x for x in rest if x not in (free, free + 1))
    return {n: FFT_MAP_DEC + 4 * x for n, x in (("beta", beta), ("mask", mask), ("free", free), ("addr", addr))}


def cx_alpha0(spec: KernelSpec) -> int:
    """First VGPR of the cx record's alpha quads: ring slots 8 and 9 (free
    from the last source chunk on), or with lds_rows (the ring is the chunk
    alone) the registers past the accumulators."""
    if spec.lds_rows:
        return spec.acc0 + 8 * spec.nacc
    return spec.ring0 + 8 * CX_ALPHA_SLOT


def cx_repair_slots(spec: KernelSpec) -> list:
    """The three ring slots the cx kernel's repair rows rotate through (the
    first two are where _fft_stream loaded rows k and k + 1; with lds_rows,
    the slots their LDS copies are read into)."""
    k, nbuf = spec.k, spec.nbuf
    ok = spec.fplan.ch == 8 and spec.k <= 64 and not getattr(spec.fplan, "direct", None) and \
        (getattr(spec.fplan, "kA", 0) or k) == k
    if spec.lds_rows:
        if not ok or nbuf != 8 or spec.ahead + 1 != spec.lds_rows:
            raise ValueError(f"{spec.name}: no cx layout")
        return [0, 1, 2]
    first = [k % nbuf, (k + 1) % nbuf]
    if not (ok and spec.ahead == 2 and nbuf == 10 and not set(first) & {CX_ALPHA_SLOT, CX_ALPHA_SLOT + 1}):
        raise ValueError(f"{spec.name}: no cx layout (power-of-two k <= 64, pd 2, chunks of 8)")
    third = next(q for q in range(nbuf) if q not in first + [CX_ALPHA_SLOT, CX_ALPHA_SLOT + 1])
    return first + [third]


def _cx_mul(E, x: list, c_reg: int, c_off: int, res: int, mt: tuple = (CX_MT, CX_MT + 1)) -> None:
    """res (8 planes) = c * x for the per-lane byte c at bits c_off.. of
    c_reg; x (8 plane registers, list by plane) is doubled in place and left
    destroyed.  8 mask extractions + 64 masked XORs + 21 doubling XORs."""
    x = list(x)
    for a in range(8):
        m = mt[a & 1]
        E(Op("v_bfe_i", (m, c_reg, c_off + a, 1)))   # all ones where bit a of c is set
        for b in range(8):
            if a == 0:
                E(Op("v_and", (res + b, x[b], m)))
            else:
                E(Op("v_xor_and", (res + b, res + b, x[b], m)))
        if a < 7:   # x <- x * 2 (poly 0x11D): bits 2, 3, 4 take bit 7; the others move up one
            for b in (1, 2, 3):
                E(Op("v_xor", (x[b], x[b], x[7])))
            x = [x[7], x[0], x[1], x[2], x[3], x[4], x[5], x[6]]


def _cx_solve(E, ops: list, spec: KernelSpec, P, fseq, load_fft, cx_slot) -> None:
    k, r, R, ch = spec.k, spec.r, P.R, P.ch
    acc0, ring0, ahead = spec.acc0, spec.ring0, spec.ahead
    n_all = len(fseq)
    planes = lambda base: [base + b for b in range(8)]
    cr = cx_regs(spec)
    # the record: beta / mask quads in the map registers the source rows no
    # longer need, alpha in ring slots 8 and 9 (free until the solve)
    E(Op("v_movs", (V_ADDR, 56)))
    E(Op("v_movs", (V_ADDR + 1, 57)))
    E(Op("v_mad64_s", (V_ADDR, V_GA, 58, V_ADDR)))
    E(Op("s_exec", (S_STA,)))
    E(Op("load16", (cr["beta"], V_ADDR, 0)))
    E(Op("load16", (cr["mask"], V_ADDR, 16)))
    alpha0 = cx_alpha0(spec)
    n_alpha = (k + 15) // 16
    for q in range(n_alpha):
        E(Op("load16", (alpha0 + 4 * q, V_ADDR, 32 + 16 * q)))
    E(Op("s_exec", (None,)))
    n_rec = 2 + n_alpha
    # loads in issue order (per-row counts), for the counted waits below
    issued = [("row", k + q, 2) for q in range(min(ahead, n_all - k))] + [("rec", None, n_rec)]

    def younger(tag):
        i = next(q for q, x in enumerate(issued) if x[:2] == tag)
        return sum(x[2] for x in issued[i + 1:])
    # accepted repairs, transposed to planes, onto their syndrome blocks
    for n in range(k, n_all):
        if n + ahead < n_all:
            load_fft(n + ahead, cx_slot(n + ahead))
            issued.append(("row", n + ahead, 2))
        E(Op("s_waitcnt_vm", (younger(("row", n)),)))
        j = fseq[n][1]
        blk0 = acc0 + 8 * P.out_block[j]
        E(Op("s_cmp_le_k_br", (S_JMAX, j, f".Lcxrep{j}")))
        base = cx_slot(n)
        if spec.lds_rows:   # the row from its LDS slot
            S = spec.lds_rows
            E(Op("ds_read_b128", (base, V_LDSA, (n % S) * LDS_ROW_BYTES)))
            E(Op("ds_read_b128", (base + 4, V_LDSA, (n % S) * LDS_ROW_BYTES + 1024)))
            E(Op("s_waitcnt_lgkm_n", (0,)))
        ops.extend(_transpose_ops(base, spec.bfi_transpose, spec.vmask))
        for b in range(8):
            E(Op("v_xor", (blk0 + b, blk0 + b, base + b)))
        E(Op("label", (f".Lcxrep{j}",)))
    E(Op("s_waitcnt_vm", (0,)))
    if spec.lab_stamps:
        E(Op("stamp", (4,)))
    # t_j = beta_j s_j; blocks of repairs no lane accepted (and of coset
    # points past r) are zero.  The products rotate through one free block:
    # block t ends in home[t]
    home = {t: acc0 + 8 * t for t in range(R)}
    free = cr["free"]
    used = set(P.out_block)
    for t in range(R):
        if t not in used:
            for b in range(8):
                E(Op("v_movk", (home[t] + b, 0)))
    for j in range(r):
        t = P.out_block[j]
        E(Op("s_cmp_le_k_br", (S_JMAX, j, f".Lcxz{j}")))
        _cx_mul(E, planes(home[t]), cr["beta"] + j // 4, 8 * (j % 4), free)
        E(Op("s_branch", (f".Lcxb{j}",)))
        E(Op("label", (f".Lcxz{j}",)))
        for b in range(8):
            E(Op("v_movk", (free + b, 0)))
        E(Op("label", (f".Lcxb{j}",)))
        home[t], free = free, home[t]
    # u = C^T t: the final butterflies transposed, in reverse
    tmp = tuple(range(V_T, V_T + 4)) if spec.fft_cse else ()
    for i, j, sc in reversed(P.final_bfly):
        for b in range(8):
            E(Op("v_xor", (home[i] + b, home[i] + b, home[j] + b)))
        if sc:
            _macc(E, home[j], home[i], sc, init=False, tmp=tmp)
    if spec.lab_stamps:
        E(Op("stamp", (5,)))
    y = [ring0 + 8 * m for m in range(ch)]
    for hc in range(k // ch):
        for m in range(ch):
            terms = P.acc[(hc, m)]
            if not terms:
                for b in range(8):
                    E(Op("v_movk", (y[m] + b, 0)))
            for q, (t, c) in enumerate(terms):
                _macc(E, y[m], home[t], c, init=q == 0, tmp=tmp)
        for i, j, sc in reversed(P.chunk_bfly[hc]):
            if sc:
                _macc(E, y[j], y[i], sc, init=False, tmp=tmp)
            for b in range(8):
                E(Op("v_xor", (y[i] + b, y[i] + b, y[j] + b)))
        for m in range(ch):
            _cx_store_row(E, ops, spec, P.order[hc * ch + m], y[m], free, alpha0, cr)


def _cx_store_row(E, ops: list, spec: KernelSpec, v: int, yreg: int, res: int, alpha0: int, cr: dict) -> None:
    """Source row v of u (planes at yreg): where a lane's generation erased
    it, x_v = alpha_v u_v to recovered row rank(v) = the erased sources
    below v; skipped when no lane of the wave erased it."""
    mw = cr["mask"] + v // 32
    skip = f".Lcxs{v}"
    E(Op("v_bfe", (V_SLOT, mw, v % 32, 1)))
    E(Op("v_cmp_ne0", (S_TMP, V_SLOT)))
    E(Op("s_nop", (4,)))
    E(Op("s_and64", (S_TMP, S_TMP, S_STA)))
    E(Op("s_cmp_eq64_0_br", (S_TMP, skip)))
    _cx_mul(E, [yreg + b for b in range(8)], alpha0 + v // 4, 8 * (v % 4), res)
    ops.extend(_transpose_ops(res, spec.bfi_transpose, spec.vmask))
    lo = v % 32
    E(Op("v_andk", (V_SLOT, (1 << lo) - 1, mw)))
    E(Op("v_bcnt0", (V_SLOT, V_SLOT)))
    if v >= 32:
        E(Op("v_bcnt", (V_SLOT, cr["mask"], V_SLOT)))
    a = cr["addr"]
    E(Op("v_mad64_s", (a, V_SLOT, 11, V_DSTA)))
    E(Op("v_add64_s", (a + 2, a, S_QB)))
    E(Op("s_and64", (S_TMP2, S_TMP, S_STA)))
    E(Op("s_exec", (S_TMP2,)))
    E(Op("store16", (a, res, 0, spec.st_policy)))
    E(Op("s_and64", (S_TMP2, S_TMP, S_STB)))
    E(Op("s_exec", (S_TMP2,)))
    E(Op("store16", (a + 2, res + 4, 0, spec.st_policy)))
    # the partial last unit: bytes [0, L % 16) of the tail lane's unit B
    E(Op("s_and64", (S_TMP2, S_TMP, S_TAIL)))
    E(Op("s_exec", (S_TMP2,)))
    E(Op("s_cbranch_execz", (f".Lcxt{v}",)))
    for b in range(15):
        E(Op("s_cmp_le_k_br", (59, b, f".Lcxt{v}")))
        E(Op("v_lshr", (V_T, 8 * (b % 4), res + 4 + b // 4)))
        E(Op("store_byte", (a + 2, V_T, b)))
        E(Op("s_nop", (0,)))
    E(Op("label", (f".Lcxt{v}",)))
    E(Op("s_exec", (None,)))
    E(Op("label", (skip,)))


def cx_record(k: int, r: int, J: list[int], E_: list[int]) -> np.ndarray:
    """The cx record of one generation (CX_REC_BYTES): beta by repair index,
    the erased-source mask, alpha by source index (zero elsewhere)."""
    from . import lch_fft
    rec = np.zeros(CX_REC_BYTES, np.uint8)
    if not E_:
        return rec
    alpha, beta = lch_fft.cauchy_inverse_factors(k, list(J), sorted(E_))
    for a, j in enumerate(J):
        rec[j] = beta[a]
    m = 0
    for b, v in enumerate(sorted(E_)):
        m |= 1 << v
        rec[32 + v] = alpha[b]
    rec[16:24] = np.frombuffer(m.to_bytes(8, "little"), np.uint8)
    return rec


def _lu_solve_and_store_chunked(E, spec: KernelSpec):
    """_lu_solve_and_store for one generation per lane: one record, 8 dwords
    per block, one split-table read per coefficient."""
    r, acc0 = spec.r, spec.acc0
    lay = lu_layout_chunked(spec)
    cols, rank, sel, tbs, tas, fp = lay["cols"], lay["rank"], lay["sel"], lay["tb"], lay["ta"], lay["fp"]
    tbx = lay.get("tbx", ((tbs[0], tbs[0] + 4), (tbs[1], tbs[1] + 4)))
    nbufs = len(tbx)
    ahead = spec.lu_ahead if spec.fft else 1
    lu = spec.lu
    bmap = spec.fplan.out_block if spec.fft else list(range(r))

    def blk(t, d):
        return acc0 + 8 * bmap[t] + d

    def store_block(t, a):
        _store_recovered_chunked(E, spec, blk, rank, t, a)

    def selectors(u):
        if spec.lu_ilp:   # stage by stage: no op depends on the one before it
            for d in range(8):
                E(Op("v_andk", (sel + d, 0x07070707, blk(u, d))))
            if spec.bfi_transpose == "s64":
                # dword pairs shifted as one 64-bit value: the bits the high
                # dword carries into the low one land in byte 3's top bits,
                # which the masks below clear
                for d in range(0, 8, 2):
                    E(Op("v_lshr64", (sel + 8 + d, 3, blk(u, d))))
                for d in range(0, 8, 2):
                    E(Op("v_lshr64", (sel + 16 + d, 6, blk(u, d))))
            else:
                for d in range(8):
                    E(Op("v_lshr", (sel + 8 + d, 3, blk(u, d))))
                for d in range(8):
                    E(Op("v_lshr", (sel + 16 + d, 6, blk(u, d))))
            for d in range(8):
                E(Op("v_andk", (sel + 8 + d, 0x07070707, sel + 8 + d)))
            for d in range(8):
                E(Op("v_andk", (sel + 16 + d, 0x03030303, sel + 16 + d)))
            return
        for d in range(8):
            x = blk(u, d)
            E(Op("v_andk", (sel + d, 0x07070707, x)))
            E(Op("v_lshr", (sel + 8 + d, 3, x)))
            E(Op("v_andk", (sel + 8 + d, 0x07070707, sel + 8 + d)))
            E(Op("v_lshr", (sel + 16 + d, 6, x)))
            E(Op("v_andk", (sel + 16 + d, 0x03030303, sel + 16 + d)))

    def table_read(u, byte, buf):
        a = tas[buf]
        tb, t2 = tbx[buf]
        E(Op("v_perm_s", (a, cols[u] + byte // 4, cols[u] + byte // 4, S_PICK + byte % 4)))
        if spec.tab_stride != 256:   # c << 8 -> c * stride
            E(Op("v_lshr", (a, 8 - (spec.tab_stride.bit_length() - 1), a)))
        E(Op("ds_read_b128", (tb, a, 0)))
        E(Op("ds_read_b32", (t2, a, 16)))

    def products(d, buf, p=(R_P, R_P + 1, R_P + 2)):
        tb, t2 = tbx[buf]
        E(Op("v_perm", (p[0], tb + 1, tb, sel + d)))
        E(Op("v_perm", (p[1], tb + 3, tb + 2, sel + 8 + d)))
        E(Op("v_perm", (p[2], t2, t2, sel + 16 + d)))

    def mul_acc(t, buf):
        if spec.lu_ilp:
            for grp in LU_ILP_GROUPS:
                for m, d in enumerate(grp):
                    products(d, buf, LU_ILP_TEMPS[3 * m: 3 * m + 3])
                for m, d in enumerate(grp):
                    E(Op("v_xor3", (blk(t, d), blk(t, d), LU_ILP_TEMPS[3 * m], LU_ILP_TEMPS[3 * m + 1])))
                for m, d in enumerate(grp):
                    E(Op("v_xor", (blk(t, d), blk(t, d), LU_ILP_TEMPS[3 * m + 2])))
            return
        for d in range(8):
            products(d, buf)
            E(Op("v_xor3", (blk(t, d), blk(t, d), R_P, R_P + 1)))
            E(Op("v_xor", (blk(t, d), blk(t, d), R_P + 2)))

    def scale(u, buf):
        if spec.lu_ilp:
            for grp in LU_ILP_GROUPS:
                for m, d in enumerate(grp):
                    products(d, buf, LU_ILP_TEMPS[3 * m: 3 * m + 3])
                for m, d in enumerate(grp):
                    E(Op("v_xor3", (blk(u, d),) + tuple(LU_ILP_TEMPS[3 * m: 3 * m + 3])))
            return
        for d in range(8):
            products(d, buf)
            E(Op("v_xor3", (blk(u, d), R_P, R_P + 1, R_P + 2)))

    def column(u, steps, end_label, guard_from):
        # table reads run `ahead` coefficients ahead of the products, in
        # nbufs = ahead + 1 rotating buffers (two LDS reads each)
        for n in range(min(ahead, len(steps))):
            table_read(u, steps[n][1], n % nbufs)
        for n, (kind, t) in enumerate(steps):
            buf = n % nbufs
            if n + ahead < len(steps):
                table_read(u, steps[n + ahead][1], (n + ahead) % nbufs)
            E(Op("s_waitcnt_lgkm_n", (2 * min(ahead, len(steps) - 1 - n),)))
            if kind == "acc":
                mul_acc(t, buf)
            else:
                scale(u, buf)
            if n + 1 < len(steps) and n + 1 >= guard_from:
                E(Op("s_cmp_le_k_br", (S_JMAX, steps[n + 1][1], end_label)))
        E(Op("label", (end_label,)))
        E(Op("s_waitcnt_lgkm_n", (0,)))

    E(Op("v_movs", (fp, 56)))
    E(Op("v_movs", (fp + 1, 57)))
    E(Op("v_mad64_s", (fp, V_GA, 58, fp)))
    E(Op("s_exec", (S_STA,)))
    for u in range(r if lu else 0):
        E(Op("load16", (cols[u], fp, 16 * u)))
    E(Op("load16", (rank, fp, 256)))
    E(Op("s_exec", (None,)))
    if lu:
        for u in range(r):
            E(Op("s_cmp_le_k_br", (S_JMAX, u, ".Lfwd_end")))
            E(Op("s_waitcnt_vm", (r - u,)))
            if spec.lab_lu_part == "bwd":
                continue
            selectors(u)
            column(u, [("scale", u)] + [("acc", t) for t in range(u + 1, r)], f".Lfwd{u}", 1)
        E(Op("label", (".Lfwd_end",)))
        if spec.lab_stamps:
            E(Op("stamp", (5,)))
        E(Op("s_waitcnt_vm", (0,)))
        pf_rows = []
        if spec.lab_prefetch:
            n_slots, _ = spec.lab_prefetch
            _prefetch_setup(E, spec)
            chunks = r - 1
            pf_rows = [list(range(n_slots))[c::chunks] for c in range(chunks)]
        for n_u, u in enumerate(reversed(range(1, r))):
            E(Op("s_cmp_le_k_br", (S_JMAX, u, f".Lbwd{u}")))
            if spec.lab_lu_part != "fwd":
                selectors(u)
                column(u, [("acc", t) for t in range(u)], f".Lbwd{u}", r + 1)
            else:
                E(Op("label", (f".Lbwd{u}",)))
            if pf_rows:
                _prefetch_rows(E, spec, len(pf_rows[n_u]))
            if spec.early_stores:
                # x_u was final before its backward column: store it now, so
                # the writes overlap the remaining columns (address in the
                # now dead column quad u)
                E(Op("s_cmp_le_k_br", (S_JMAX, u, f".Lstu{u}")))
                E(Op("s_nop", (4,)))
                store_block(u, cols[u])
                E(Op("label", (f".Lstu{u}",)))
        if spec.lab_prefetch:
            E(Op("label", (".Lnopf",)))
        if spec.early_stores:
            E(Op("s_cmp_le_k_br", (S_JMAX, 0, ".Lst_end")))
            E(Op("s_nop", (4,)))
            store_block(0, cols[0])
            E(Op("label", (".Lst_end",)))
            return
    else:
        E(Op("s_waitcnt_vm", (0,)))
    # stores: block t -> recovered row rank[t]; A half, then B half at + 16 Q
    E(Op("s_nop", (4,)))
    st = [c for c in cols]     # column quads are dead now: store address pairs
    na = 0
    for t in range(r):
        E(Op("s_cmp_le_k_br", (S_JMAX, t, ".Lst_end")))
        a = st[na % len(st)]
        na += 1
        store_block(t, a)
    E(Op("label", (".Lst_end",)))


def _store_recovered_chunked(E, spec: KernelSpec, blk, rank: int, t: int, a: int):
    """Block t (byte form) -> recovered row rank[t] of the lane's generation:
    A half at the lane's unit q, B half at + 16 Q, the partial last unit
    bytewise (a, a + 2: address pairs)."""
    E(Op("v_bfe", (V_SLOT, rank + t // 4, 8 * (t % 4), 8)))
    E(Op("v_cmp_ne_s", (S_TMP, S_ABSENT, V_SLOT)))
    E(Op("s_nop", (4,)))
    E(Op("v_mad64_s", (a, V_SLOT, 11, V_DSTA)))
    E(Op("v_add64_s", (a + 2, a, S_QB)))
    E(Op("s_and64", (S_TMP2, S_TMP, S_STA)))
    E(Op("s_exec", (S_TMP2,)))
    E(Op("store16", (a, blk(t, 0), 0, spec.st_policy)))
    E(Op("s_and64", (S_TMP2, S_TMP, S_STA if spec.lab_full_b_store else S_STB)))
    E(Op("s_exec", (S_TMP2,)))
    E(Op("store16", (a + 2, blk(t, 4), 0, spec.st_policy)))
    # the partial last unit: bytes [0, L % 16) of the tail lane's unit B
    E(Op("s_and64", (S_TMP2, S_TMP, S_TAIL)))
    E(Op("s_exec", (S_TMP2,)))
    E(Op("s_cbranch_execz", (f".Ltl{t}",)))
    for b in range(15):
        E(Op("s_cmp_le_k_br", (59, b, f".Ltl{t}")))
        E(Op("v_lshr", (V_T, 8 * (b % 4), blk(t, 4 + b // 4))))
        E(Op("store_byte", (a + 2, V_T, b)))
        E(Op("s_nop", (0,)))
    E(Op("label", (f".Ltl{t}",)))
    E(Op("s_exec", (None,)))


# --------------------------------------------------------------------------
# Bit-sliced payload pass with wave-uniform runtime coefficients ("cmb")
# --------------------------------------------------------------------------
# x_E = D s for the decode paths' k_combine_slots records (one 16-byte record
# of 16 output coefficients per input row and pass), one generation per item:
# item = (g, t), lanes q = 64 t + l < Q own units q and q + Q of each row
# (Q = ceil(Lu / 2)), so every coefficient is wave-uniform.  Per input row:
# 8 bit planes (transpose), their 4-bit combinations LO[0..15] / HI[0..15]
# (LO[0] = HI[0] = 0), then per output j
#     acc_j[p] ^= LO[M_c row p & 15];  acc_j[p] ^= HI[M_c row p >> 4]
# with the register chosen by the scalar unit: s_set_gpr_idx_{on,idx} and a
# v_xor_b32 whose src0 is M0-indexed, the 16 indices of c read as one
# s_load_dwordx16 from a 256 x 64-byte table (cmb_index_table).
# tools/ubench_idx.py: 16 indexed XORs + 17 index writes issue at about half
# the plain XOR rate, against 24 v_perm + 8 v_bitop3 per product in
# k_combine_slots.
#
# kernarg (128 bytes, s4..s35):
#   s[4:5] rows  s[6:7] dst  s[8:9] rows gen stride  s[10:11] dst gen stride
#   s12 row stride  s13 dst row stride  s[14:15] coefficient records
#   s16 record gen stride  s17 pass  s[18:19] n_out  s[20:21] bound
#   s[22:23] index table  s[24:25] rows offset table  s[26:27] dst offset table
#   s28 L  s29 Lu  s30 Q  s31 items per generation  s32 items  s33 grid waves
#   s34 / s35 magic / shift of the division by s31
KERNARG_BYTES_CMB = 128
CMB_NEXT_FREE_VGPR = 192
CMB_NEXT_FREE_SGPR = 102
C_OA, C_OB = 2, 3                 # lane byte offsets of units A / B in a row
C_BUF = (4, 12)                   # two 8-dword row buffers (A: +0..3, B: +4..7)
C_T = 20                          # v20..v23 transpose temps
C_LO, C_HI = 24, 40               # LO[0..15], HI[0..15]
C_ACC = 56                        # 16 x 8 accumulators v56..v183
C_QV, C_QC, C_UB, C_UBC, C_TB = 184, 185, 186, 187, 188
C_VM = 189                        # v189..v191 transpose masks (full-rate all-VGPR v_bitop3)
CMB_WIDE_R = 24                   # the wide single pass: outputs 16..23 from the pass-1 record


def _cmb_regs(R: int) -> dict:
    """VGPRs past the accumulators: the fixed layout above for R <= 16; the
    wide pass (R = 24, 192 accumulators) moves them above its accumulators
    (256 VGPRs: still two waves per SIMD)."""
    if 8 < R <= 16:
        return {"qv": C_QV, "qc": C_QC, "ub": C_UB, "ubc": C_UBC, "tb": C_TB, "vm": C_VM, "end": CMB_NEXT_FREE_VGPR}
    # R <= 8: 128 VGPRs (four waves per SIMD); R = 24: 256 (two)
    b = C_ACC + 8 * R
    return {"qv": b, "qc": b + 1, "ub": b + 2, "ubc": b + 3, "tb": b + 4, "vm": b + 5, "end": b + 8}
# SGPRs
CS_ITEM, CS_G, CS_T, CS_EW, CS_BOUND, CS_SLOT = 36, 37, 38, 39, 40, 41
CS_ROWG, CS_CUR, CS_NEXT, CS_COEFG, CS_DSTG = 42, 44, 46, 48, 50
CS_REC = 52                       # s52..s55 (4-aligned for s_load_dwordx4)
CS_IDX = (56, 72)                 # two 16-SGPR index buffers (4-aligned)
CS_VALID, CS_FULLB, CS_TAIL, CS_TMP64 = 88, 90, 92, 94
CS_MASKS = 96                     # s96..s98 transpose masks
CS_T0, CS_T1, CS_TBYTES = 99, 100, 3
# wide pass (R > 16): s[0:1] the pass-1 record's first 8 bytes (outputs 16..23),
# s2 its offset (free once the kernarg is loaded and the workgroup id read),
# s101 the records' pass stride (kernarg word 32)
CS_REC2, CS_REC2_OFF, CS_PSTRIDE = 0, 2, 101


def cmb_index_table() -> np.ndarray:
    """256 x 16 dwords: for coefficient c and output plane p, dword 2p = the
    LO index (row p of M_c, input planes 0-3) and 2p + 1 = the HI index."""
    t = np.zeros((256, 16), np.uint32)
    for c in range(256):
        rows = mul_matrix_rows(c)
        for p in range(8):
            t[c, 2 * p], t[c, 2 * p + 1] = rows[p] & 15, rows[p] >> 4
    return t


def _cmb_transpose(E, base: int, last_dst: Optional[list] = None, vm0: int = C_VM):
    """bfi delta-swap network on 8 registers (plane p <- bit p of every byte);
    the last stage writes plane p to last_dst[p] (default: in place)."""
    for stage, (sh, _mask, pairs) in enumerate(_TRANSPOSE):
        vm = vm0 + stage
        for q, (a, b) in enumerate(pairs):
            t, u = C_T + 2 * (q & 1), C_T + 2 * (q & 1) + 1
            da, db = base + a, base + b
            if stage == 2 and last_dst is not None:
                da, db = last_dst[a], last_dst[b]
            E(Op("v_lshl", (t, sh, base + b)))
            E(Op("v_lshr", (u, sh, base + a)))
            E(Op("v_bitsel_v", (da, vm, base + a, t)))
            E(Op("v_bitsel_v", (db, vm, u, base + b)))


def _cmb_gen_addr(E, dst: int, base: int, gs: int, offs: int, tag: str):
    """s[dst:dst+1] <- base + g * gen_stride (64-bit stride s[gs:gs+1]), or
    base + offs[g] when the offset table pointer is non-zero."""
    E(Op("s_cmp_eq64_0_br", (offs, f".Lcs{tag}")))
    E(Op("s_lshl", (CS_T0, CS_G, 3)))
    E(Op("s_load_n", (CS_TMP64, offs, 2, CS_T0, 0)))
    E(Op("s_waitcnt_lgkm", ()))
    E(Op("s_branch", (f".Lca{tag}",)))
    E(Op("label", (f".Lcs{tag}",)))
    E(Op("s_mul", (CS_TMP64, CS_G, gs)))            # lo(g * gs_lo)
    E(Op("s_mul_hi", (CS_TMP64 + 1, CS_G, gs)))     # hi(g * gs_lo)
    E(Op("s_mul", (CS_T0, CS_G, gs + 1)))
    E(Op("s_add", (CS_TMP64 + 1, CS_TMP64 + 1, CS_T0)))
    E(Op("label", (f".Lca{tag}",)))
    E(Op("s_add_cc", (dst, base, CS_TMP64)))
    E(Op("s_addc", (dst + 1, base + 1, CS_TMP64 + 1)))


def _cmb_row(E, spec, buf: int, other: int, tag: str):
    """One input row (slot CS_SLOT, data in `buf`): prefetch the next row into
    `other`, bit-slice, combinations, then the ew products."""
    E(Op("s_lshl", (CS_T0, CS_SLOT, 4)))
    if spec.pass_major and spec.r == CMB_WIDE_R:
        # pm24: outputs 8t..8t+7 of the pass from the record byte offset D_t
        # (s22 / s23 / s101, _cmb_pm24_prologue), three 8-byte pieces
        for dst, d, tmp in ((CS_REC, PM24_D[0], CS_REC2_OFF), (CS_REC + 2, PM24_D[1], PM24_T[0]),
                            (CS_REC2, PM24_D[2], PM24_T[1])):
            E(Op("s_add", (tmp, CS_T0, d)))
            E(Op("s_load_n", (dst, CS_COEFG, 2, tmp, 0)))
    else:
        E(Op("s_load_n", (CS_REC, CS_COEFG, 4, CS_T0, 0)))
    if spec.r > 16 and not spec.pass_major:   # outputs 16.. from the pass-1 record of the row
        E(Op("s_add", (CS_REC2_OFF, CS_T0, CS_PSTRIDE)))
        E(Op("s_load_n", (CS_REC2, CS_COEFG, 2, CS_REC2_OFF, 0)))
    ahead = 2 if spec.cmb_pf2 else 1
    E(Op("s_addk", (CS_T0, CS_SLOT, ahead)))
    E(Op("s_cmp_ge_br", (CS_T0, CS_BOUND, f".Lnopf{tag}")))
    if spec.cmb_pf2:   # CS_NEXT: the last row issued
        E(Op("s_add_cc", (CS_NEXT, CS_NEXT, 12)))
        E(Op("s_addck", (CS_NEXT + 1, CS_NEXT + 1, 0)))
    else:
        E(Op("s_add_cc", (CS_NEXT, CS_CUR, 12)))
        E(Op("s_addck", (CS_NEXT + 1, CS_CUR + 1, 0)))
    if "noload" not in spec.lab_cmb:
        E(Op("load16_saddr", (other, C_OA, CS_NEXT, spec.ld_policy)))
        E(Op("load16_saddr", (other + 4, C_OB, CS_NEXT, spec.ld_policy)))
    E(Op("s_waitcnt_vm", (2 * ahead,)))
    E(Op("s_branch", (f".Lrow{tag}",)))
    E(Op("label", (f".Lnopf{tag}",)))
    E(Op("s_waitcnt_vm", (0,)))
    E(Op("label", (f".Lrow{tag}",)))
    singles = [C_LO + 1, C_LO + 2, C_LO + 4, C_LO + 8, C_HI + 1, C_HI + 2, C_HI + 4, C_HI + 8]
    _cmb_transpose(E, buf, singles, _cmb_regs(spec.r)["vm"])
    for tab in (C_LO, C_HI):
        for m in sorted(_COMBO_BUILD):
            a, b = _COMBO_BUILD[m]
            E(Op("v_xor", (tab + m, tab + a, tab + b)))
    E(Op("s_waitcnt_lgkm", ()))
    if not spec.cmb_jump:   # index rows of output 0's coefficient
        E(Op("s_bfe_k", (CS_T0, CS_REC, 0, 8)))
        E(Op("s_lshl", (CS_T0, CS_T0, 6)))
        E(Op("s_load_n", (CS_IDX[0], 22, 16, CS_T0, 0)))
    def rec_sgpr(j: int) -> int:   # the SGPR holding output j's coefficient byte
        return CS_REC + j // 4 if j < 16 else CS_REC2 + (j - 16) // 4

    lean = spec.cmb_lean
    if spec.cmb_jump:
        _cmb_jump_products(E, spec, rec_sgpr, tag)
        return
    for j in range(spec.r):
        if j and (not lean or j % 4 == 0):
            E(Op("s_cmp_le_k_br", (CS_EW, j, f".Lpe{tag}")))
        E(Op("s_waitcnt_lgkm", ()))
        if j + 1 < spec.r and "idx_once" not in spec.lab_cmb:   # the next output's indices load during this product
            E(Op("s_bfe_k", (CS_T0, rec_sgpr(j + 1), 8 * ((j + 1) % 4), 8)))
            E(Op("s_lshl", (CS_T0, CS_T0, 6)))
            E(Op("s_load_n", (CS_IDX[(j + 1) % 2], 22, 16, CS_T0, 0)))
        ix = CS_IDX[0] if "idx_once" in spec.lab_cmb else CS_IDX[j % 2]
        for p in range(8):
            acc = C_ACC + 8 * j + p
            E(Op("s_idx_on" if p == 0 and (j == 0 or not lean) else "s_idx", (ix + 2 * p,)))
            E(Op("v_xor_rel", (acc, C_LO, acc)))
            E(Op("s_idx", (ix + 2 * p + 1,)))
            E(Op("v_xor_rel", (acc, C_HI, acc)))
        if not lean:
            E(Op("s_idx_off", ()))
    E(Op("label", (f".Lpe{tag}",)))
    if lean:   # every exit leaves after product 0, with the mode on
        E(Op("s_idx_off", ()))
    E(Op("s_waitcnt_lgkm", ()))


# jump products: 8 j by output (s56..s79, the index-row buffers' SGPRs), the
# call target, the return address, the table's address
CJ_J8, CJ_TGT, CJ_RET, CJ_TAB = 56, 80, 82, 84
CJ_BLOCK = 128                                   # bytes per coefficient block (a power of two)
CJ_FAKE_TAB = 0x7F0000000000                     # the emulator's table address


def _cmb_jump_products(E, spec: KernelSpec, rec_sgpr, tag: str):
    """Row products as calls into the coefficient blocks (KernelSpec.cmb_jump):
    index 8 j on the destination (and the accumulator source), block c =
    output j's record byte; every 4 outputs the early exit (lean)."""
    assert spec.r <= 24 and spec.cmb_lean and CJ_J8 + spec.r <= CJ_TGT
    E(Op("s_idx_on_d3" if spec.cmb_jump == 3 else "s_idx_on_d2", (CJ_J8,)))
    for j in range(spec.r):
        if j and j % 4 == 0:
            E(Op("s_cmp_le_k_br", (CS_EW, j, f".Lpe{tag}")))
        if j:
            E(Op("s_idx", (CJ_J8 + j,)))
        E(Op("s_bfe_k", (CS_T0, rec_sgpr(j), 8 * (j % 4), 8)))
        E(Op("s_lshl", (CS_T0, CS_T0, CJ_BLOCK.bit_length() - 1)))
        E(Op("s_add_cc", (CJ_TGT, CJ_TAB, CS_T0)))
        E(Op("s_addck", (CJ_TGT + 1, CJ_TAB + 1, 0)))
        E(Op("s_call", (CJ_RET, CJ_TGT)))
    E(Op("label", (f".Lpe{tag}",)))
    E(Op("s_idx_off", ()))


def _cmb_jump_table(E, spec: KernelSpec):
    """After s_endpgm: the 256 coefficient blocks, CJ_BLOCK bytes apart from
    .Ltab (acc_j[p] ^= LO[row p of M_c & 15] ^ HI[row p >> 4], j by gpr_idx)."""
    tab = cmb_index_table()
    E(Op("align7", ()))
    E(Op("label", (".Ltab",)))
    for c in range(256):
        E(Op("label", (f".Lblk{c}",)))
        for p in range(8):
            a, b = int(tab[c, 2 * p]), int(tab[c, 2 * p + 1])
            if spec.cmb_jump == 3:
                E(Op("v_xor3_reld", (C_ACC + p, C_LO + a, C_HI + b)))
            else:
                E(Op("v_xor_reld", (C_ACC + p, C_LO + a)))
                E(Op("v_xor_reld", (C_ACC + p, C_HI + b)))
        E(Op("s_ret", (CJ_RET,)))
        E(Op("align7", ()))


# pm24 (24-output pass-major, jump products only): the three record pieces'
# byte offsets (the index-row SGPRs s22:23, dead in jump mode, and s101) and
# the address temps (free in jump mode)
PM24_D = (22, 23, 101)
PM24_T = (86, 87)


def _cmb_pm24_prologue(E):
    """Pass p' of a 24-output pass-major launch (workgroups [p' n, (p' + 1) n),
    at most 3 passes): outputs 24 p' .. 24 p' + 23 are the 16-output record
    passes' bytes [24 p', 24 p' + 24), i.e. record pass q0 = (3 p') >> 1 from
    byte 8 (p' & 1), in three 8-byte pieces at D_t = 8 (p' & 1) + 8 t past
    pass q0 (a piece past 15 is the next record pass's, D - 16 + pass
    stride). Pieces in a record pass that was not written (q0 + 1 >= word 33)
    read piece 0 instead: their outputs lie past e_max and are never stored.
    The coefficient base advances by q0 record passes, the output rows by
    24 p' rows."""
    E(Op("s_lshrk", (CS_TMP64 + 1, 33, 2)))            # n = workgroups per pass
    E(Op("s_movk", (17, 0)))
    for _ in range(2):
        E(Op("s_cmp_lt_br", (2, CS_TMP64 + 1, ".Lpm_done")))
        E(Op("s_sub", (2, 2, CS_TMP64 + 1)))
        E(Op("s_addk", (17, 17, 1)))
        E(Op("s_mul_k", (CS_TMP64, 13, CMB_WIDE_R)))   # dst += 24 rows
        E(Op("s_add_cc", (6, 6, CS_TMP64)))
        E(Op("s_addck", (7, 7, 0)))
    E(Op("label", (".Lpm_done",)))
    # q0 = (3 p') >> 1 record passes: p' = 1 -> 1, p' = 2 -> 3
    E(Op("s_mul_k", (36, 17, 3)))
    E(Op("s_lshrk", (36, 36, 1)))
    E(Op("s_movk", (37, 0)))
    E(Op("label", (".Lpm_q",)))
    E(Op("s_cmp_ge_br", (37, 36, ".Lpm_qd")))
    E(Op("s_addk", (37, 37, 1)))
    E(Op("s_add_cc", (14, 14, CS_T1)))
    E(Op("s_addck", (15, 15, 0)))
    E(Op("s_branch", (".Lpm_q",)))
    E(Op("label", (".Lpm_qd",)))
    # D0 = 8 (p' & 1); D1 = p' odd ? stride : 8; D2 = p' odd ? stride + 8 : stride
    # (D2 takes s101, word 33: the record-pass count moves to s41 first)
    E(Op("s_mov", (41, CS_T1 + 1)))
    E(Op("s_andk", (38, 17, 1)))
    E(Op("s_lshl", (PM24_D[0], 38, 3)))
    E(Op("s_movk", (39, 8)))
    E(Op("s_add", (40, CS_T1, 39)))                    # stride + 8
    E(Op("s_cmp_eq_k", (38, 1)))
    E(Op("s_cselect32", (PM24_D[1], CS_T1, 39)))
    E(Op("s_cselect32", (PM24_D[2], 40, CS_T1)))
    # record pass q0 + 1 not written: its pieces read piece 0
    E(Op("s_addk", (36, 36, 1)))
    E(Op("s_cmp_lt_br", (36, 41, ".Lpm_dok")))
    E(Op("s_mov", (PM24_D[2], PM24_D[0])))
    E(Op("s_cmp_eq_k", (38, 1)))
    E(Op("s_cselect32", (PM24_D[1], PM24_D[0], PM24_D[1])))
    E(Op("label", (".Lpm_dok",)))


def _generate_cmb(spec: KernelSpec) -> list[Op]:
    ops: list[Op] = []
    E = ops.append
    R = spec.r
    assert R <= 16 or (R == CMB_WIDE_R and (not spec.pass_major or (spec.cmb_jump and not spec.pm_xcd)))
    pm24 = spec.pass_major and R == CMB_WIDE_R
    rg = _cmb_regs(R)
    C_QV, C_QC, C_UB, C_UBC, C_TB, C_VM = (rg[x] for x in ("qv", "qc", "ub", "ubc", "tb", "vm"))
    assert C_ACC + 8 * R <= C_QV and rg["end"] <= 256
    E(Op("s_load_n", (4, 0, 16, None, 0)))
    E(Op("s_load_n", (20, 0, 16, None, 64)))
    E(Op("v_lshr", (1, 6, 0)))
    E(Op("v_andk", (0, 63, 0)))
    E(Op("v_readfirstlane", (CS_T0, 1)))
    for q, (_, mask, _) in enumerate(_TRANSPOSE):
        E(Op("s_movk", (CS_MASKS + q, mask)))
        E(Op("v_movs", (C_VM + q, CS_MASKS + q)))
    E(Op("v_movk", (C_LO, 0)))
    E(Op("v_movk", (C_HI, 0)))
    if spec.cmb_jump:
        assert spec.cmb_jump in (2, 3) and 8 * 8 + 4 <= CJ_BLOCK   # 8 VOP3 or 16 VOP2 + the return
        E(Op("s_getpc_rel", (CJ_TAB, ".Ltab")))
        for j in range(R):
            E(Op("s_movk", (CJ_J8 + j, 8 * j)))
    assert not spec.pm_xcd or spec.pass_major
    if spec.pm_xcd:   # records' pass stride; word 33: (magic << 3) | passes
        E(Op("s_load_n", (CS_T1, 0, 2, None, KERNARG_BYTES_CMB)))
    elif pm24:        # records' pass stride; word 33: the record passes written
        E(Op("s_load_n", (CS_T1, 0, 2, None, KERNARG_BYTES_CMB)))
    elif spec.pass_major:
        E(Op("s_load_n", (CS_T1, 0, 1, None, KERNARG_BYTES_CMB)))   # records' pass stride
    if R > 16 and not pm24:
        E(Op("s_load_n", (CS_PSTRIDE, 0, 1, None, KERNARG_BYTES_CMB)))
    E(Op("s_waitcnt_lgkm", ()))
    if spec.pm_xcd:
        # workgroup w = 8 h + x: pass p = h mod P, slot 8 (h div P) + x, with
        # h div P = (h * ceil(2^16 / P)) >> 16 (exact for h < 2^15, P <= 4)
        E(Op("s_andk", (36, 2, 7)))                  # x
        E(Op("s_lshrk", (37, 2, 3)))                 # h
        E(Op("s_lshrk", (38, CS_T1 + 1, 3)))         # magic
        E(Op("s_andk", (39, CS_T1 + 1, 7)))          # P
        E(Op("s_mul", (40, 37, 38)))
        E(Op("s_lshrk", (40, 40, 16)))               # q = h div P
        E(Op("s_mul", (41, 40, 39)))
        E(Op("s_sub", (41, 37, 41)))                 # p = h - q P
        E(Op("s_lshl", (2, 40, 3)))
        E(Op("s_add", (2, 2, 36)))                   # the slot
        E(Op("s_movk", (17, 0)))
        for _ in range(3):
            E(Op("s_cmp_ge_br", (17, 41, ".Lpm_done")))
            E(Op("s_addk", (17, 17, 1)))
            E(Op("s_add", (14, 14, CS_T1)))
            E(Op("s_addck", (15, 15, 0)))
            E(Op("s_lshl", (CS_TMP64, 13, 4)))
            E(Op("s_add", (6, 6, CS_TMP64)))
            E(Op("s_addck", (7, 7, 0)))
        E(Op("label", (".Lpm_done",)))
    elif pm24:
        _cmb_pm24_prologue(E)
    elif spec.pass_major:
        # workgroups [p n, (p + 1) n) run pass p (n = grid waves / 4): the
        # pass, its records and its 16 output rows, and the workgroup id in
        # the pass's range (at most 4 passes: e <= 64)
        # (CS_T0 holds the wave's index in its workgroup: n goes to s95)
        E(Op("s_lshrk", (CS_TMP64 + 1, 33, 2)))
        E(Op("s_movk", (17, 0)))
        for _ in range(3):
            E(Op("s_cmp_lt_br", (2, CS_TMP64 + 1, ".Lpm_done")))
            E(Op("s_sub", (2, 2, CS_TMP64 + 1)))
            E(Op("s_addk", (17, 17, 1)))
            E(Op("s_add", (14, 14, CS_T1)))
            E(Op("s_addck", (15, 15, 0)))
            E(Op("s_lshl", (CS_TMP64, 13, 4)))
            E(Op("s_add", (6, 6, CS_TMP64)))
            E(Op("s_addck", (7, 7, 0)))
        E(Op("label", (".Lpm_done",)))
    E(Op("s_lshl", (CS_ITEM, 2, 2)))
    E(Op("s_add", (CS_ITEM, CS_ITEM, CS_T0)))
    E(Op("s_andk", (CS_TBYTES, 28, 15)))            # L % 16: bytes of a partial last unit
    E(Op("label", (".Litem",)))
    E(Op("s_cmp_lt_br", (CS_ITEM, 32, ".Lgo")))
    E(Op("s_branch", (".Lend",)))
    E(Op("label", (".Lgo",)))
    # g = item / ipg (ipg == 1: g = item), t = item - g ipg
    E(Op("s_mul_hi", (CS_G, CS_ITEM, 34)))
    E(Op("s_lshr_s", (CS_G, CS_G, 35)))
    E(Op("s_cmp_eq_k", (31, 1)))
    E(Op("s_cselect32", (CS_G, CS_ITEM, CS_G)))
    E(Op("s_mul", (CS_T0, CS_G, 31)))
    E(Op("s_sub", (CS_T, CS_ITEM, CS_T0)))
    E(Op("s_lshl", (CS_T0, CS_G, 2)))
    E(Op("s_load_n", (CS_T1, 18, 1, CS_T0, 0)))      # e = n_out[g]
    E(Op("s_load_n", (CS_BOUND, 20, 1, CS_T0, 0)))   # bound[g]
    E(Op("s_waitcnt_lgkm", ()))
    # outputs of this pass: ew = min(e - 16 pass, R) (24 pass for pm24); none -> next item
    if pm24:
        E(Op("s_mul_k", (CS_T0, 17, CMB_WIDE_R)))
    else:
        E(Op("s_lshl", (CS_T0, 17, 4)))
    E(Op("s_cmp_ge_br", (CS_T0, CS_T1, ".Lnext")))
    E(Op("s_sub", (CS_EW, CS_T1, CS_T0)))
    E(Op("s_movk", (CS_T0, R)))
    E(Op("s_min", (CS_EW, CS_EW, CS_T0)))
    _cmb_gen_addr(E, CS_ROWG, 4, 8, 24, "r")
    _cmb_gen_addr(E, CS_DSTG, 6, 10, 26, "d")
    E(Op("s_mul", (CS_TMP64, CS_G, 16)))
    E(Op("s_mul_hi", (CS_TMP64 + 1, CS_G, 16)))
    E(Op("s_add_cc", (CS_COEFG, 14, CS_TMP64)))
    E(Op("s_addc", (CS_COEFG + 1, 15, CS_TMP64 + 1)))
    # lanes: qv = 64 t + l; valid = qv < Q; qc = min(qv, Q - 1); ub = qc + Q
    E(Op("v_lshl_add_s", (C_QV, CS_T, 6, 0)))
    E(Op("v_cmp_gt_s", (CS_VALID, 30, C_QV)))
    E(Op("s_addk", (CS_T0, 30, -1)))
    E(Op("v_min_s", (C_QC, CS_T0, C_QV)))
    E(Op("v_add_s", (C_UB, 30, C_QC)))
    E(Op("v_cmp_gt_s", (CS_FULLB, 29, C_UB)))        # ub < Lu
    E(Op("s_addk", (CS_T0, 29, -1)))
    E(Op("v_min_s", (C_UBC, CS_T0, C_UB)))
    E(Op("v_cmp_eq_s", (CS_TAIL, CS_T0, C_UB)))      # ub == Lu - 1
    E(Op("s_nop", (4,)))
    E(Op("s_and64", (CS_FULLB, CS_FULLB, CS_VALID)))
    E(Op("s_and64", (CS_TAIL, CS_TAIL, CS_FULLB)))
    E(Op("s_movk", (CS_TMP64, 0)))
    E(Op("s_movk", (CS_TMP64 + 1, 0)))
    E(Op("s_cmp_eq_k", (CS_TBYTES, 0)))
    E(Op("s_cselect64", (CS_TAIL, CS_TMP64, CS_TAIL)))   # whole last unit: no tail lane
    E(Op("s_andn2_64", (CS_FULLB, CS_FULLB, CS_TAIL)))
    E(Op("v_lshl", (C_OA, 4, C_QC)))
    E(Op("v_lshl", (C_OB, 4, C_UBC)))
    for a in range(C_ACC, C_ACC + 8 * R):
        E(Op("v_movk", (a, 0)))
    # input rows, two per loop trip (ring of two row buffers)
    E(Op("s_movk", (CS_SLOT, 0)))
    E(Op("s_mov", (CS_CUR, CS_ROWG)))
    E(Op("s_mov", (CS_CUR + 1, CS_ROWG + 1)))
    E(Op("s_cmp_le_k_br", (CS_BOUND, 0, ".Lstores")))
    E(Op("load16_saddr", (C_BUF[0], C_OA, CS_CUR, spec.ld_policy)))
    E(Op("load16_saddr", (C_BUF[0] + 4, C_OB, CS_CUR, spec.ld_policy)))
    bufs = list(C_BUF)
    if spec.cmb_pf2:   # row 1 in flight too; CS_NEXT tracks the last row issued
        assert R <= 16
        bufs.append(rg["end"])
        E(Op("s_mov", (CS_NEXT, CS_CUR)))
        E(Op("s_mov", (CS_NEXT + 1, CS_CUR + 1)))
        E(Op("s_cmp_le_k_br", (CS_BOUND, 1, ".Lpf1")))
        E(Op("s_add_cc", (CS_NEXT, CS_NEXT, 12)))
        E(Op("s_addck", (CS_NEXT + 1, CS_NEXT + 1, 0)))
        E(Op("load16_saddr", (bufs[1], C_OA, CS_NEXT, spec.ld_policy)))
        E(Op("load16_saddr", (bufs[1] + 4, C_OB, CS_NEXT, spec.ld_policy)))
        E(Op("label", (".Lpf1",)))
    nb = len(bufs)
    ahead = 2 if spec.cmb_pf2 else 1
    E(Op("label", (".Lslot",)))
    for h in range(nb):
        _cmb_row(E, spec, bufs[h], bufs[(h + ahead) % nb], f"{h}")
        E(Op("s_addk", (CS_SLOT, CS_SLOT, 1)))
        E(Op("s_cmp_ge_br", (CS_SLOT, CS_BOUND, ".Lstores")))
        if not spec.cmb_pf2:
            E(Op("s_mov", (CS_CUR, CS_NEXT)))
            E(Op("s_mov", (CS_CUR + 1, CS_NEXT + 1)))
    E(Op("s_branch", (".Lslot",)))
    # recovered rows: bytes back (inverse transpose), unit A on valid lanes,
    # unit B where it is a whole unit, and the partial last unit bytewise
    E(Op("label", (".Lstores",)))
    for j in range(R):
        acc = C_ACC + 8 * j
        E(Op("s_cmp_le_k_br", (CS_EW, j, ".Lst_end")))
        _cmb_transpose(E, acc, None, C_VM)
        E(Op("s_movk", (CS_T0, j)))
        E(Op("s_mul", (CS_T0, CS_T0, 13)))
        E(Op("s_add_cc", (CS_TMP64, CS_DSTG, CS_T0)))
        E(Op("s_addck", (CS_TMP64 + 1, CS_DSTG + 1, 0)))
        E(Op("s_exec", (CS_VALID,)))
        E(Op("store16_saddr", (C_OA, acc, CS_TMP64, spec.st_policy)))
        E(Op("s_exec", (CS_FULLB,)))
        E(Op("store16_saddr", (C_OB, acc + 4, CS_TMP64, spec.st_policy)))
        E(Op("s_exec", (CS_TAIL,)))
        E(Op("s_cbranch_execz", (f".Ltl{j}",)))
        for b in range(15):
            E(Op("s_cmp_le_k_br", (CS_TBYTES, b, f".Ltl{j}")))
            E(Op("v_lshr", (C_TB, 8 * (b % 4), acc + 4 + b // 4)))
            E(Op("store_byte_saddr", (C_OB, C_TB, CS_TMP64, b)))
            E(Op("s_nop", (0,)))
        E(Op("label", (f".Ltl{j}",)))
        E(Op("s_exec", (None,)))
        E(Op("s_nop", (1,)))   # store data registers are not rewritten right after the store
    E(Op("label", (".Lst_end",)))
    E(Op("label", (".Lnext",)))
    E(Op("s_nop", (4,)))
    E(Op("s_add", (CS_ITEM, CS_ITEM, 33)))
    E(Op("s_branch", (".Litem",)))
    E(Op("label", (".Lend",)))
    E(Op("s_endpgm", ()))
    if spec.cmb_jump:
        _cmb_jump_table(E, spec)
    return ops


def pm_xcd_word(passes: int) -> int:
    """Kernarg word 33 of the interleaved pass-major payload kernel
    (KernelSpec.pm_xcd): (ceil(2^16 / P) << 3) | P."""
    assert 2 <= passes <= 4
    return (-(-65536 // passes) << 3) | passes


def cmb_kernargs(rows: int, dst: int, rgs: int, dgs: int, rs: int, drs: int, coef: int, cgs: int, pas: int,
                 n_out: int, bound: int, idxtab: int, L: int, G: int, total_waves: int,
                 rows_offs: int = 0, dst_offs: int = 0, pass_stride: Optional[int] = None,
                 pm_xcd_passes: int = 0) -> tuple[bytes, int]:
    """Kernarg block of qf_combine_bs (layout above) and the item count;
    pass_stride: the pass-major kernel's word 32 (records of pass p at
    coef + p pass_stride, its outputs at dst + 16 p drs); pm_xcd_passes: the
    interleaved pass-major kernel's pass count (word 33, pm_xcd_word)."""
    Lu = (L + 15) // 16
    Q = (Lu + 1) // 2
    ipg = (Q + 63) // 64
    magic, shift = magic_for(ipg) if ipg >= 2 else (0, 0)
    n_items = G * ipg
    words = [rows & MASK32, rows >> 32, dst & MASK32, dst >> 32, rgs & MASK32, rgs >> 32, dgs & MASK32, dgs >> 32,
             rs, drs, coef & MASK32, coef >> 32, cgs, pas, n_out & MASK32, n_out >> 32, bound & MASK32,
             bound >> 32, idxtab & MASK32, idxtab >> 32, rows_offs & MASK32, rows_offs >> 32,
             dst_offs & MASK32, dst_offs >> 32, L, Lu, Q, ipg, n_items, total_waves, magic, shift]
    if pass_stride is not None:
        words += [pass_stride, pm_xcd_word(pm_xcd_passes) if pm_xcd_passes else 0]
    for w in words:
        assert 0 <= w < 1 << 32, words
    return np.array(words, np.uint32).tobytes(), n_items


# --------------------------------------------------------------------------
# Assembly text
# --------------------------------------------------------------------------
def emit_asm(spec: KernelSpec, ops: list[Op]) -> str:
    name = spec.name
    body = []
    for op in ops:
        s = op.asm()
        if op.name == "label":
            body.append(s.replace(".L", f".L{name}_"))
        else:
            body.append("\t" + s.replace(".L", f".L{name}_"))
    nv = spec.next_free_vgpr
    meta_args = [
        ("src", 0, 8, "global_buffer"), ("dst", 8, 8, "global_buffer"),
    ]
    args_yaml = []
    for nm, off, sz, kind in meta_args:
        args_yaml.append(f"""      - .address_space:  global
        .name:           {nm}
        .offset:         {off}
        .size:           {sz}
        .value_kind:     {kind}""")
    args_yaml.append(f"""      - .name:           params
        .offset:         16
        .size:           {spec.kernarg_bytes - 16}
        .value_kind:     by_value""")
    return f"""\t.amdgcn_target "amdgcn-amd-amdhsa--gfx950"
\t.amdhsa_code_object_version 6
\t.text
\t.globl\t{name}
\t.p2align\t8
\t.type\t{name},@function
{name}:
""" + "\n".join(body) + f"""
\t.section\t.rodata,"a",@progbits
\t.p2align\t6, 0x0
\t.amdhsa_kernel {name}
\t\t.amdhsa_group_segment_fixed_size {spec.lds_bytes}
\t\t.amdhsa_private_segment_fixed_size 0
\t\t.amdhsa_kernarg_size {spec.kernarg_bytes}
\t\t.amdhsa_user_sgpr_count 2
\t\t.amdhsa_user_sgpr_kernarg_segment_ptr 1
\t\t.amdhsa_system_sgpr_workgroup_id_x 1
\t\t.amdhsa_system_vgpr_workitem_id 0
\t\t.amdhsa_next_free_vgpr {nv}
\t\t.amdhsa_next_free_sgpr {spec.next_free_sgpr}
\t\t.amdhsa_accum_offset {nv}
\t\t.amdhsa_reserve_vcc 0
\t\t.amdhsa_float_denorm_mode_32 3
\t\t.amdhsa_float_denorm_mode_16_64 3
\t.end_amdhsa_kernel
\t.text
.Lfunc_end_{name}:
\t.size\t{name}, .Lfunc_end_{name}-{name}

\t.amdgpu_metadata
---
amdhsa.kernels:
  - .args:
{chr(10).join(args_yaml)}
    .group_segment_fixed_size: {spec.lds_bytes}
    .kernarg_segment_align: 8
    .kernarg_segment_size: {spec.kernarg_bytes}
    .max_flat_workgroup_size: {64 * getattr(spec, "waves", 4)}
    .name:           {name}
    .private_segment_fixed_size: 0
    .sgpr_count:     {spec.next_free_sgpr + 6}
    .sgpr_spill_count: 0
    .symbol:         {name}.kd
    .vgpr_count:     {nv}
    .vgpr_spill_count: 0
    .wavefront_size: 64
    .agpr_count:     0
amdhsa.target:   amdgcn-amd-amdhsa--gfx950
amdhsa.version:
  - 1
  - 2
...
\t.end_amdgpu_metadata
"""


# --------------------------------------------------------------------------
# Host-side launch parameters
# --------------------------------------------------------------------------
def magic_for(U: int) -> tuple[int, int]:
    """g = mulhi(f, magic) >> shift == f // U for f < 2**31 (U >= 2)."""
    s = (U - 1).bit_length()  # 2**(s-1) < U <= 2**s
    magic = -(-(1 << (31 + s)) // U)
    assert magic < (1 << 32)
    return magic, s - 1


def padded_units(L: int) -> int:
    """Lane units per row that align items to 128-B lines: ceil(L/16) rounded up to 8."""
    return ((L + 15) // 16 + 7) // 8 * 8


def tail_masks(L: int) -> list[int]:
    """Per-dword byte masks of a row's last 16-B unit (enc kernarg words 16..19):
    bytes < L % 16 kept, all ones when L % 16 == 0."""
    tb = L % 16 or 16
    return [MASK32 if tb - 4 * d >= 4 else (1 << (8 * max(0, tb - 4 * d))) - 1 for d in range(4)]


def launch_geometry(L: int, G: int, Lv: Optional[int] = None) -> tuple[int, int, int]:
    """(Lv, total units, items) of a batch: 16-byte units, 128 per item, Lv
    lane units per row (default ceil(L/16); L % 16 != 0 needs the zero-tail
    lane space)."""
    if L < 32 or (L % 16 and Lv is None):
        raise ValueError("bit-sliced kernels need L >= 32, and the zero tail when L % 16 != 0")
    Lu = (L + 15) // 16
    Lv = Lu if Lv is None else Lv
    if Lv < Lu:
        raise ValueError("Lv < L/16")
    total = G * Lv
    if total >= 1 << 31:
        raise ValueError("too many units for one launch")
    return Lv, total, (total + 127) // 128


def kernargs(src: int, dst: int, sgs: int, dgs: int, srs: int, drs: int, L: int, G: int,
             total_waves: int, smap: int = 0, map_stride: int = 0, zero: int = 0,
             Lv: Optional[int] = None, zero_tail: bool = False, lu: Optional[tuple[int, int]] = None,
             tables: int = 0, src_offs: int = 0, dst_offs: int = 0, chunked: bool = False,
             bound: Optional[int] = None, wave_gen: bool = False, Q: Optional[int] = None) -> bytes:
    """96-byte kernarg block (layout above; 128 bytes in dec mode).  Syndrome mode: src = received
    rows, dst = syndrome rows, plus slot map and zero row.  zero_tail (enc):
    also write zeros to bytes [L, 16 Lv) of every repair row.  Dec mode
    (lu = (records, record stride), tables = split-table base): dst, dgs and
    drs are the recovered rows' base, generation and row strides; 112 bytes."""
    Lv, total, n_items = launch_geometry(L, G, Lv)
    magic, shift = magic_for(Lv)
    if chunked:   # lane-chunk layout (_prologue_chunked): Lv <- Q = ceil(Lu / 2) (Q: a larger one)
        Lv = ((L + 15) // 16 + 1) // 2
        if Q is not None:
            assert Lv <= Q < (L + 15) // 16
            Lv = Q
        total = G * Lv
        n_items = G if wave_gen else (total + 63) // 64
        magic, shift = magic_for(Lv)
    s19 = map_stride if smap else (Lv if zero_tail else L // 16)
    if L % 16 and not (zero_tail or smap):
        raise ValueError("enc with L % 16 != 0 needs the zero tail")
    tail = [smap & MASK32, smap >> 32, zero & MASK32, zero >> 32] if smap else tail_masks(L)
    words = [src & MASK32, src >> 32, dst & MASK32, dst >> 32, sgs, dgs, srs, drs, (L + 15) // 16, Lv, total,
             magic, shift, n_items, total_waves, s19] + tail
    if lu is not None:   # word 23: L % 16 (the lane-chunk decode's partial last unit)
        words += [lu[0] & MASK32, lu[0] >> 32, lu[1], (L % 16) if chunked else 0, tables & MASK32, tables >> 32, 0, 0]
    # generation offset tables (0: strided generations)
    words += [src_offs & MASK32, src_offs >> 32, dst_offs & MASK32, dst_offs >> 32]
    if bound is not None:   # synw: per-generation pass bound table (0: none)
        words += [bound & MASK32, bound >> 32]
    for w in words:
        assert 0 <= w < 1 << 32, words
    return np.array(words, dtype=np.uint32).tobytes()


def perm_record(c: int) -> list[int]:
    """gf256_tables.h perm_record: {T0lo, T0hi, T1lo, T1hi, T2, 0, 0, 0}."""
    t0 = [gf_mul(c, v) for v in range(8)]
    t1 = [gf_mul(c, v << 3) for v in range(8)]
    t2 = [gf_mul(c, v << 6) for v in range(4)]

    def pk(b):
        return b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24
    return [pk(t0[:4]), pk(t0[4:]), pk(t1[:4]), pk(t1[4:]), pk(t2), 0, 0, 0]


def split_tables() -> np.ndarray:
    """The 256 x 32-byte table set the dec kernel copies into LDS."""
    return np.array([perm_record(c) for c in range(256)], np.uint32).reshape(-1).view(np.uint8)


def lu_record(k: int, r: int, accepted: list[int], E: list[int]) -> np.ndarray:
    """Host restatement of k_decode_prepare_lu's per-generation record: the
    LU factors (no pivoting) of A = C[J, E] with J = accepted repairs
    ascending and E = erased sources ascending (U with unit diagonal after
    dividing each row by its pivot; the pivots' inverses on the diagonal),
    embedded by repair index
    (LU_REC_BYTES bytes; layout in _lu_solve_and_store).  Every leading minor
    of a Cauchy matrix is non-zero, so the factorisation needs no pivoting."""
    J = sorted(accepted)
    e = len(J)
    assert e == len(E) and e <= 16 and r <= 16
    A = [[gf_inv(((k + j) & 0xFF) ^ i) for i in E] for j in J]
    Lm = [[0] * e for _ in range(e)]
    for p in range(e):
        inv = gf_inv(A[p][p])
        for i in range(p + 1, e):
            f = gf_mul(A[i][p], inv)
            Lm[i][p] = f
            for c in range(p, e):
                A[i][c] ^= gf_mul(f, A[p][c])
    rec = np.zeros(LU_REC_BYTES, np.uint8)
    rec[256:272] = 0xFF
    for b, t in enumerate(J):
        rec[256 + t] = b
        for c, u in enumerate(J):
            if b < c:
                v = gf_mul(A[b][c], gf_inv(A[b][b]))    # U'[b][c] = U[b][c] / U[b][b]
            elif b == c:
                v = gf_inv(A[b][b])
            else:
                v = Lm[b][c]
            rec[16 * u + t] = v
    return rec


def cauchy_inverse(k: int, J: list[int], E: list[int]) -> list[list[int]]:
    """D = C[J, E]^-1 in closed form (rows: erased sources E, columns: the
    accepted repairs J in the given order).  With X_a = k + J[a] and
    Y_b = E[b] (all distinct, k + r <= 256):
      D[b][a] = A_a B_b / ((X_a + Y_b) E_a F_b),  A_a = prod_t (X_a + Y_t),
      B_b = prod_t (X_t + Y_b), E_a = prod_{t!=a} (X_a + X_t),
      F_b = prod_{t!=b} (Y_b + Y_t)."""
    X = [(k + j) & 0xFF for j in J]
    Y = list(E)
    e = len(X)

    def lg(v):
        return _LOG[v]
    lA = [sum(lg(X[a] ^ Y[t]) for t in range(e)) for a in range(e)]
    lB = [sum(lg(X[t] ^ Y[b]) for t in range(e)) for b in range(e)]
    lE = [sum(lg(X[a] ^ X[t]) for t in range(e) if t != a) for a in range(e)]
    lF = [sum(lg(Y[b] ^ Y[t]) for t in range(e) if t != b) for b in range(e)]
    return [[_EXP[(lA[a] + lB[b] - lg(X[a] ^ Y[b]) - lE[a] - lF[b]) % 255] for a in range(e)]
            for b in range(e)]


# --------------------------------------------------------------------------
# Emulator (64 lanes, one wave at a time) -- test infrastructure
# --------------------------------------------------------------------------
class EmuError(RuntimeError):
    pass


class Emulator:
    """Executes the IR for every wave of a grid against a flat byte memory.

    Loads are asynchronous: their destination registers are marked pending
    until an s_waitcnt vmcnt(n) retires them in issue order; reading a pending
    register raises.  Every access is bounds-checked against the registered
    buffers."""

    def __init__(self, ops: list[Op]):
        self.ops = ops
        self.labels = {op.args[0]: n for n, op in enumerate(ops) if op.name == "label"}
        self.buffers: list[tuple[int, int]] = []
        self.mem = {}
        self.executed = {}   # op name -> times executed (over every wave run): dynamic instruction counts

    def add_buffer(self, base: int, data: np.ndarray):
        self.buffers.append((base, len(data)))
        self.mem[base] = data

    def _find(self, addr: int, n: int):
        for base, size in self.buffers:
            if base <= addr and addr + n <= base + size:
                return base
        raise EmuError(f"out-of-bounds access 0x{addr:x}+{n}")

    def read(self, addr: int, n: int) -> bytes:
        b = self._find(addr, n)
        return self.mem[b][addr - b: addr - b + n].tobytes()

    def write(self, addr: int, data: bytes):
        b = self._find(addr, len(data))
        self.mem[b][addr - b: addr - b + len(data)] = np.frombuffer(data, np.uint8)

    def run_wave(self, kernarg: bytes, workgroup: int, wave_in_wg: int):
        """One wave alone (an s_barrier lets it through at once)."""
        gen = self._wave(kernarg, workgroup, wave_in_wg, None)
        while True:
            try:
                next(gen)
            except StopIteration as e:
                return e.value

    def run_workgroup(self, kernarg: bytes, workgroup: int, n_waves: int, lds_bytes: int):
        """The waves of one workgroup over one shared LDS: each runs to its
        next s_barrier (or its end) in turn, and a barrier releases once every
        wave still running has reached it (waves that ended do not count, as
        on the hardware)."""
        lds = np.zeros(lds_bytes, np.uint8)
        gens = {w: self._wave(kernarg, workgroup, w, lds) for w in range(n_waves)}
        steps = 0
        while gens:
            for w in list(gens):
                try:
                    next(gens[w])
                except StopIteration as e:
                    steps += e.value
                    del gens[w]
        return steps

    def _wave(self, kernarg: bytes, workgroup: int, wave_in_wg: int, shared_lds):
        v = np.zeros((256, 64), dtype=np.uint64)
        s = [0] * 104
        lds = np.zeros(160 * 1024, np.uint8) if shared_lds is None else shared_lds
        m0_lds = 0
        lds_busy = {}     # LDS byte ranges with an LDS-DMA outstanding: id -> (lo, hi)
        pend_lgkm = []
        ka = np.frombuffer(kernarg, np.uint32)
        pending = []  # list of (regs, values, lanes) in issue order
        busy = set()
        busy_lanes = {}   # load16_saddr: register -> lanes with a load outstanding
        exec_ = np.ones(64, bool)
        tid = np.arange(64, dtype=np.uint64) + 64 * wave_in_wg
        v[0] = tid
        s[2] = workgroup

        def rv(i):
            if i in busy or (i in busy_lanes and busy_lanes[i].any()):
                raise EmuError(f"read of v{i} with a load outstanding")
            return v[i]

        def wv(i, val):
            if i in busy:
                raise EmuError(f"write of v{i} with a load outstanding")
            v[i] = np.where(exec_, np.asarray(val, dtype=np.uint64) & MASK32, v[i])

        def rv64(i):
            return rv(i) | (rv(i + 1) << np.uint64(32))

        def wv64(i, val):
            val = np.asarray(val, dtype=np.uint64)
            wv(i, val & np.uint64(MASK32))
            wv(i + 1, val >> np.uint64(32))

        def smask(i):
            m = s[i] | (s[i + 1] << 32)
            return np.array([(m >> l) & 1 for l in range(64)], bool)

        def set_smask(i, arr):
            m = 0
            for l in range(64):
                if arr[l]:
                    m |= 1 << l
            s[i], s[i + 1] = m & MASK32, m >> 32

        pc = 0
        ops = self.ops
        scc = 0
        steps = 0
        pend_s = []        # s_load_n: (first SGPR, values) written at the next lgkmcnt(0)
        idx_mode, m0 = False, 0
        idx_dst, call_ret = False, None   # gpr_idx on the destination (jump products); the open call

        def retire_s():
            for d0, w in pend_s:
                for q, x in enumerate(w):
                    s[d0 + q] = int(x)
            pend_s.clear()

        while True:
            op = ops[pc]
            pc += 1
            steps += 1
            n, a = op.name, op.args
            self.executed[n] = self.executed.get(n, 0) + 1
            if idx_mode and n.startswith("v_") and n not in ("v_xor_rel", "v_xor3_reld", "v_xor_reld"):
                raise EmuError(f"{n} while the gpr_idx mode is on")
            if n == "s_waitcnt_lgkm" or (n == "s_waitcnt_lgkm_n" and a[0] == 0):
                retire_s()
            if n in ("label", "s_nop", "s_waitcnt_lgkm", "s_setprio", "s_stagger", "stamp", "align7"):
                continue
            if n == "s_load_args":
                for q in range(20):
                    s[4 + q] = int(ka[q])
            elif n == "s_load_args_dec":
                for q in range(8):
                    s[56 + q] = int(ka[20 + q])
            elif n == "s_load_args_offs":
                for q in range(4):
                    s[72 + q] = int(ka[a[0] // 4 + q])
            elif n == "s_cmp_eq64_0_br":
                if s[a[0]] == 0 and s[a[0] + 1] == 0:
                    pc = self.labels[a[1]]
            elif n == "load8":
                d, ar, off = a
                addr = rv64(ar)
                vals = np.zeros((2, 64), np.uint64)
                for l in np.nonzero(exec_)[0]:
                    vals[:, l] = np.frombuffer(self.read(int(addr[l]) + off, 8), np.uint32)
                regs = [d, d + 1]
                for rg in regs:
                    if rg in busy:
                        raise EmuError(f"load into v{rg} with a load outstanding")
                    busy.add(rg)
                pending.append((regs, vals, exec_.copy()))
            elif n == "v_add64_v":
                wv64(a[0], rv64(a[1]) + rv64(a[2]))
            elif n in ("v_perm", "v_perm_s"):
                pool = (rv(a[1]) << np.uint64(32)) | rv(a[2])
                sel = rv(a[3]) if n == "v_perm" else np.full(64, s[a[3]], np.uint64)
                res = np.zeros(64, np.uint64)
                for b in range(4):
                    sb = (sel >> np.uint64(8 * b)) & np.uint64(0xFF)
                    if ((sb >= 8) & (sb != 12)).any():
                        raise EmuError("v_perm selector outside 0..7, 12")
                    byte = np.where(sb == 12, np.uint64(0),
                                    (pool >> (np.minimum(sb, 7) * np.uint64(8))) & np.uint64(0xFF))
                    res |= byte << np.uint64(8 * b)
                wv(a[0], res)
            elif n == "s_m0":
                m0_lds = (s[a[0]] + a[1]) & MASK32
            elif n == "load16_lds":
                addr = rv64(a[0])
                base = m0_lds
                if base < 0 or base + 1024 > len(lds):
                    raise EmuError(f"LDS-DMA out of range 0x{base:x}")
                buf = np.zeros(1024, np.uint8)
                wmask = np.zeros(1024, bool)
                for l in np.nonzero(exec_)[0]:
                    buf[16 * l: 16 * l + 16] = np.frombuffer(self.read(int(addr[l]), 16), np.uint8)
                    wmask[16 * l: 16 * l + 16] = True
                key = object()
                lds_busy[key] = (base, base + 1024)
                pending.append((("lds", key, base, buf, wmask), None, None))
            elif n in ("ds_read_b128", "ds_read_b32"):
                d, ar, off = a
                nd = 4 if n == "ds_read_b128" else 1
                addr = rv(ar)
                vals = np.zeros((nd, 64), np.uint64)
                for l in np.nonzero(exec_)[0]:
                    p0 = int(addr[l]) + off
                    if p0 < 0 or p0 + 4 * nd > len(lds):
                        raise EmuError(f"LDS access out of range 0x{p0:x}")
                    for lo_, hi_ in lds_busy.values():
                        if p0 < hi_ and p0 + 4 * nd > lo_:
                            raise EmuError(f"ds_read of LDS 0x{p0:x} with an LDS-DMA outstanding")
                    vals[:, l] = np.frombuffer(lds[p0: p0 + 4 * nd].tobytes(), np.uint32)
                regs = [d + q for q in range(nd)]
                for rg in regs:
                    if rg in busy:
                        raise EmuError(f"ds_read into v{rg} with a load outstanding")
                    busy.add(rg)
                pend_lgkm.append((regs, vals, exec_.copy()))
            elif n == "ds_write_b128":
                ar, d, off = a
                addr = rv(ar)
                vals = np.stack([rv(d + q) for q in range(4)]).astype(np.uint32)
                for l in np.nonzero(exec_)[0]:
                    p0 = int(addr[l]) + off
                    if p0 < 0 or p0 + 16 > len(lds):
                        raise EmuError(f"LDS access out of range 0x{p0:x}")
                    lds[p0: p0 + 16] = np.frombuffer(vals[:, l].tobytes(), np.uint8)
            elif n == "s_waitcnt_lgkm_n":
                while len(pend_lgkm) > a[0]:
                    regs, vals, lanes = pend_lgkm.pop(0)
                    for q, rg in enumerate(regs):
                        busy.discard(rg)
                        v[rg] = np.where(lanes, vals[q], v[rg])
            elif n == "s_cmp_le_k_br":
                if s[a[0]] <= a[1]:
                    pc = self.labels[a[2]]
            elif n == "s_or64":
                set_smask(a[0], smask(a[1]) | smask(a[2]))
            elif n == "s_cmp_lg64_br":
                if s[a[0]] or s[a[0] + 1]:
                    pc = self.labels[a[1]]
            elif n == "v_xor":
                wv(a[0], rv(a[1]) ^ rv(a[2]))
            elif n == "v_mov":
                wv(a[0], rv(a[1]))
            elif n == "v_xor3":
                wv(a[0], rv(a[1]) ^ rv(a[2]) ^ rv(a[3]))
            elif n == "v_bitsel_s":
                m = np.uint64(s[a[1]])
                wv(a[0], (m & rv(a[2])) | (~m & np.uint64(MASK32) & rv(a[3])))
            elif n == "v_bitsel_v":
                m = rv(a[1])
                wv(a[0], (m & rv(a[2])) | (~m & np.uint64(MASK32) & rv(a[3])))
            elif n == "v_movk":
                wv(a[0], np.full(64, a[1], np.uint64))
            elif n == "v_andk":
                wv(a[0], rv(a[2]) & np.uint64(a[1]))
            elif n == "v_lshr":
                wv(a[0], rv(a[2]) >> np.uint64(a[1]))
            elif n == "v_lshl":
                wv(a[0], (rv(a[2]) << np.uint64(a[1])) & np.uint64(MASK32))
            elif n == "v_lshl64":
                wv64(a[0], rv64(a[2]) << np.uint64(a[1]))
            elif n == "v_lshr64":
                wv64(a[0], rv64(a[2]) >> np.uint64(a[1]))
            elif n == "v_lshr_s":
                wv(a[0], rv(a[2]) >> np.uint64(s[a[1]] & 31))
            elif n == "v_addk":
                wv(a[0], (rv(a[2]) + np.uint64(a[1])) & np.uint64(MASK32))
            elif n == "v_add_s":
                wv(a[0], (rv(a[2]) + np.uint64(s[a[1]])) & np.uint64(MASK32))
            elif n == "v_sub":
                wv(a[0], (rv(a[1]) - rv(a[2])) & np.uint64(MASK32))
            elif n == "v_lshl_add_s":
                wv(a[0], ((np.uint64(s[a[1]]) << np.uint64(a[2])) + rv(a[3])) & np.uint64(MASK32))
            elif n == "v_mul_hi_s":
                wv(a[0], (rv(a[1]) * np.uint64(s[a[2]])) >> np.uint64(32))
            elif n == "v_mul_lo_s":
                wv(a[0], (rv(a[1]) * np.uint64(s[a[2]])) & np.uint64(MASK32))
            elif n == "v_movs":
                wv(a[0], np.full(64, s[a[1]], np.uint64))
            elif n == "v_mad64_s":
                wv64(a[0], rv(a[1]) * np.uint64(s[a[2]]) + rv64(a[3]))
            elif n == "v_mad64_k":
                wv64(a[0], rv(a[1]) * np.uint64(a[2]) + rv64(a[3]))
            elif n == "v_add64_s":
                wv64(a[0], rv64(a[1]) + np.uint64(s[a[2]] | (s[a[2] + 1] << 32)))
            elif n in ("v_cmp_gt_s", "v_cmp_ge_s"):
                x = rv(a[2])
                sv = np.uint64(s[a[1]])
                res = (sv > x) if n == "v_cmp_gt_s" else (sv >= x)
                set_smask(a[0], res & exec_)
            elif n == "v_readfirstlane":
                lane = int(np.argmax(exec_))
                s[a[0]] = int(rv(a[1])[lane])
            elif n == "v_bfe":
                wv(a[0], (rv(a[1]) >> np.uint64(a[2])) & np.uint64((1 << a[3]) - 1))
            elif n == "v_bfe_i":
                f = (rv(a[1]) >> np.uint64(a[2])) & np.uint64((1 << a[3]) - 1)
                sign = (f >> np.uint64(a[3] - 1)) & np.uint64(1)
                wv(a[0], np.where(sign == 1, f | (np.uint64(MASK32) ^ np.uint64((1 << a[3]) - 1)), f))
            elif n == "v_and":
                wv(a[0], rv(a[1]) & rv(a[2]))
            elif n == "v_xor_and":
                wv(a[0], rv(a[1]) ^ (rv(a[2]) & rv(a[3])))
            elif n in ("v_bcnt0", "v_bcnt"):
                x = rv(a[1]).astype(np.uint64)
                cnt = np.array([bin(int(q)).count("1") for q in x], np.uint64)
                wv(a[0], (cnt + (rv(a[2]) if n == "v_bcnt" else np.uint64(0))) & np.uint64(MASK32))
            elif n == "v_cmp_ne0":
                set_smask(a[0], (rv(a[1]) != 0) & exec_)
            elif n == "v_cmp_ne_s":
                set_smask(a[0], (rv(a[2]) != np.uint64(s[a[1]])) & exec_)
            elif n == "v_cmp_eq_s":
                set_smask(a[0], (rv(a[2]) == np.uint64(s[a[1]])) & exec_)
            elif n == "v_and_s":
                wv(a[0], rv(a[2]) & np.uint64(s[a[1]]))
            elif n == "s_cmp_eq_k_br":
                if s[a[0]] == a[1]:
                    pc = self.labels[a[2]]
            elif n == "s_cmp_lg_k_br":
                if s[a[0]] != a[1]:
                    pc = self.labels[a[2]]
            elif n == "s_cbranch_execz":
                if not exec_.any():
                    pc = self.labels[a[0]]
            elif n == "v_cndmask":
                wv(a[0], np.where(smask(a[3]), rv(a[2]), rv(a[1])))
            elif n == "load16":
                d, ar, off = a[:3]
                addr = rv64(ar)
                vals = np.zeros((4, 64), np.uint64)
                lanes = np.nonzero(exec_)[0]
                for l in lanes:
                    raw = self.read(int(addr[l]) + off, 16)
                    vals[:, l] = np.frombuffer(raw, np.uint32)
                regs = [d + q for q in range(4)]
                for rg in regs:
                    if rg in busy:
                        raise EmuError(f"load into v{rg} with a load outstanding")
                    busy.add(rg)
                pending.append((regs, vals, exec_.copy()))
            elif n == "store16":
                ar, d, off = a[:3]
                addr = rv64(ar)
                vals = np.stack([rv(d + q) for q in range(4)]).astype(np.uint32)
                for l in np.nonzero(exec_)[0]:
                    self.write(int(addr[l]) + off, vals[:, l].tobytes())
            elif n == "s_waitcnt_vm":
                while len(pending) > a[0]:
                    regs, vals, lanes = pending.pop(0)
                    if regs[0] == "lds":      # an LDS-DMA lands
                        _, key, base, buf, wmask = regs
                        seg = lds[base: base + 1024]
                        seg[wmask] = buf[wmask]
                        del lds_busy[key]
                        continue
                    for q, rg in enumerate(regs):
                        busy.discard(rg)
                        if rg in busy_lanes:
                            busy_lanes[rg] &= ~lanes
                        v[rg] = np.where(lanes, vals[q], v[rg])
            elif n == "load16_saddr":
                d, voff, sb = a[:3]
                base = s[sb] | (s[sb + 1] << 32)
                off = rv(voff)
                vals = np.zeros((4, 64), np.uint64)
                for l in np.nonzero(exec_)[0]:
                    vals[:, l] = np.frombuffer(self.read(base + int(off[l]), 16), np.uint32)
                regs = [d + q for q in range(4)]
                for rg in regs:
                    bl = busy_lanes.setdefault(rg, np.zeros(64, bool))
                    if rg in busy or (bl & exec_).any():
                        raise EmuError(f"load into v{rg} lanes with a load outstanding")
                    bl |= exec_
                pending.append((regs, vals, exec_.copy()))
            elif n == "s_load_karg_x2":
                s[a[0]], s[a[0] + 1] = int(ka[a[1] // 4]), int(ka[a[1] // 4 + 1])
            elif n in ("s_load_x1", "s_load_x2", "s_load_x4"):
                d, ar, off = a
                nd = {"s_load_x1": 1, "s_load_x2": 2, "s_load_x4": 4}[n]
                addr = (s[ar] | (s[ar + 1] << 32)) + off
                if addr % 4:
                    raise EmuError("unaligned scalar load")
                w = np.frombuffer(self.read(addr, 4 * nd), np.uint32)
                for q in range(nd):
                    s[d + q] = int(w[q])
            elif n == "s_addk":
                t = s[a[1]] + (a[2] & MASK32)
                s[a[0]], scc = t & MASK32, int(t > MASK32)
            elif n == "s_add_cc":
                t = s[a[1]] + s[a[2]]
                s[a[0]], scc = t & MASK32, int(t > MASK32)
            elif n == "s_addc":
                t = s[a[1]] + s[a[2]] + scc
                s[a[0]], scc = t & MASK32, int(t > MASK32)
            elif n == "s_addck":
                t = s[a[1]] + (a[2] & MASK32) + scc
                s[a[0]], scc = t & MASK32, int(t > MASK32)
            elif n == "s_mul_hi":
                s[a[0]] = (s[a[1]] * s[a[2]]) >> 32
            elif n == "s_max":
                s[a[0]] = max(s[a[1]], s[a[2]])
            elif n == "s_lshr_s":
                s[a[0]] = s[a[1]] >> (s[a[2]] & 31)
            elif n == "s_bfe_k":
                s[a[0]] = (s[a[1]] >> a[2]) & ((1 << a[3]) - 1)
            elif n == "s_cmp_eq_k":
                scc = int(s[a[0]] == a[1])
            elif n == "s_cselect64":
                src = a[1] if scc else a[2]
                s[a[0]], s[a[0] + 1] = s[src], s[src + 1]
            elif n == "s_exec":
                exec_ = np.ones(64, bool) if a[0] is None else smask(a[0])
            elif n == "s_and64":
                set_smask(a[0], smask(a[1]) & smask(a[2]))
            elif n == "s_andn2_64":
                set_smask(a[0], smask(a[1]) & ~smask(a[2]))
            elif n == "s_mov":
                s[a[0]] = s[a[1]]
            elif n == "s_movk":
                s[a[0]] = a[1] & MASK32
            elif n == "s_add":
                s[a[0]] = (s[a[1]] + s[a[2]]) & MASK32
            elif n == "s_lshl":
                s[a[0]] = (s[a[1]] << a[2]) & MASK32
            elif n == "s_lshrk":
                s[a[0]] = s[a[1]] >> a[2]
            elif n == "s_andk":
                s[a[0]] = s[a[1]] & a[2]
            elif n == "s_mul":
                s[a[0]] = (s[a[1]] * s[a[2]]) & MASK32
            elif n == "s_mul_k":
                s[a[0]] = (s[a[1]] * a[2]) & MASK32
            elif n == "s_ashr31":
                s[a[0]] = MASK32 if s[a[1]] >> 31 else 0
            elif n == "s_min":
                s[a[0]] = min(s[a[1]], s[a[2]])
            elif n == "s_cmp_ge_br":
                if s[a[0]] >= s[a[1]]:
                    pc = self.labels[a[2]]
            elif n == "s_branch" or n == "s_far_jump":
                pc = self.labels[a[0]]
            elif n == "s_cmp_lt_br":
                if s[a[0]] < s[a[1]]:
                    pc = self.labels[a[2]]
            elif n == "s_load_n":
                d, base, nd, soff, imm = a
                if base == 0:   # s[0:1]: the kernarg segment
                    pend_s.append((d, ka[imm // 4: imm // 4 + nd].copy()))
                    continue
                addr = (s[base] | (s[base + 1] << 32)) + (s[soff] if soff is not None else 0) + imm
                if addr % 4:
                    raise EmuError("unaligned scalar load")
                pend_s.append((d, np.frombuffer(self.read(addr, 4 * nd), np.uint32).copy()))
            elif n == "s_sub":
                t = s[a[1]] - s[a[2]]
                s[a[0]], scc = t & MASK32, int(t < 0)
            elif n == "s_cselect32":
                s[a[0]] = s[a[1]] if scc else s[a[2]]
            elif n == "v_min_s":
                wv(a[0], np.minimum(rv(a[2]), np.uint64(s[a[1]])))
            elif n in ("s_idx_on", "s_idx", "s_idx_on_d3", "s_idx_on_d2"):
                if n == "s_idx" and not idx_mode:
                    raise EmuError("s_set_gpr_idx_idx outside the gpr_idx mode")
                if n != "s_idx":
                    idx_dst = n != "s_idx_on"
                idx_mode, m0 = True, s[a[0]] & 0xFF
            elif n == "s_getpc_rel":
                s[a[0]], s[a[0] + 1] = CJ_FAKE_TAB & MASK32, CJ_FAKE_TAB >> 32
            elif n == "s_call":
                if call_ret is not None:
                    raise EmuError("nested s_swappc")
                off = (s[a[1]] | (s[a[1] + 1] << 32)) - CJ_FAKE_TAB
                if off % CJ_BLOCK or not 0 <= off < 256 * CJ_BLOCK:
                    raise EmuError(f"call outside the coefficient table (offset {off})")
                s[a[0]], s[a[0] + 1] = 0xC0DE, 0
                call_ret, pc = pc, self.labels[f".Lblk{off // CJ_BLOCK}"]
            elif n == "s_ret":
                if call_ret is None or s[a[0]] != 0xC0DE:
                    raise EmuError("s_setpc without a call")
                pc, call_ret = call_ret, None
            elif n in ("v_xor3_reld", "v_xor_reld"):
                if not (idx_mode and idx_dst):
                    raise EmuError(f"{n} outside the destination gpr_idx mode")
                d = a[0] + m0
                if d >= 256:
                    raise EmuError(f"indexed destination v{d}")
                x = rv(d) ^ rv(a[1])
                wv(d, x ^ rv(a[2]) if n == "v_xor3_reld" else x)
            elif n == "s_idx_off":
                idx_mode = False
            elif n == "v_xor_rel":
                if not idx_mode or idx_dst:
                    raise EmuError("v_xor_rel outside the gpr_idx mode")
                wv(a[0], rv(a[1] + m0) ^ rv(a[2]))
            elif n == "store_byte":
                addr = rv64(a[0])
                val = rv(a[1])
                for l in np.nonzero(exec_)[0]:
                    self.write(int(addr[l]) + a[2], bytes([int(val[l]) & 0xFF]))
            elif n in ("store16_saddr", "store_byte_saddr"):
                voff, d, sb = a[:3]
                base = s[sb] | (s[sb + 1] << 32)
                off = rv(voff)
                for l in np.nonzero(exec_)[0]:
                    if n == "store16_saddr":
                        self.write(base + int(off[l]),
                                   np.array([rv(d + q)[l] for q in range(4)], np.uint32).tobytes())
                    else:
                        self.write(base + int(off[l]) + a[3], bytes([int(rv(d)[l]) & 0xFF]))
            elif n == "stamp_flush":   # lab_stamps: 72 B at stamps + 128 item (pointer: kernarg bytes 128..135)
                pending.clear()
                base = int(ka[KERNARG_BYTES_DEC // 4]) | (int(ka[KERNARG_BYTES_DEC // 4 + 1]) << 32)
                self.write(base + 128 * s[28], bytes(72))
            elif n == "s_barrier":
                if pend_lgkm:
                    raise EmuError("s_barrier with LDS operations outstanding")
                yield steps
            elif n == "s_endpgm":
                if pending:
                    # stores/loads may be outstanding at the end: retire them
                    pending.clear()
                return steps
            else:
                raise EmuError(f"unknown op {n}")
