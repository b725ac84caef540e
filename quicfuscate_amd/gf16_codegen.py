"""Bit-sliced GF(2^16) Cauchy encode kernels (HIP C++ generated per (k, r)).

The reference's GF(2^16) repair coefficients are a fixed Cauchy matrix per
(k, r): C[j][i] = gf16_inv(i ^ (k + j)) (decoder.rs:77-80, SURVEY F2 field
0x1100B).  Multiplication by a fixed c is a fixed GF(2)-linear map of the 16
symbol bits, so, as for GF(2^8) (bs_codegen.py), each product becomes XORs of
bit planes with compile-time operands and no table lookups:

* a lane owns 4 units of 16 B of a row (units q, q + Q, q + 2Q, q + 3Q of its
  generation, Q = ceil(Lu / 4)): 16 dwords = 32 big-endian symbols;
* a 4-stage delta-swap network (an involution) turns the 16 dwords into 16
  planes: after it, register b holds raw bit b of every symbol half-word
  (raw bit b is symbol bit (b + 8) % 16: the symbols are big-endian);
* the planes are split into 4 groups of 4; the 15 XOR combinations of each
  group are formed once per row (44 XORs), so every output plane of every
  product is the XOR of at most 4 combination registers (2 v_xor3: groups
  {0, 1}, then {2, 3}, so 22 combinations are live at a time);
* an empty asm with the accumulators as operands closes every row, so the
  compiler does not reassociate the XOR chains across rows and keeps one
  row's temporaries live (the next row's loads are issued before it);
* 8 repairs per pass (8 x 16 accumulator planes); passes re-read the rows.

`generate(k, r)` returns C++ source text (kernel qf_gf16bs_k{k}_r{r}, all passes);
`emulate(k, r, rows)` runs the same term lists on numpy arrays (the CPU test
compares it with the oracle), and `terms(k, r)` exposes the schedule.
"""
from __future__ import annotations

import functools

import numpy as np

POLY = 0x1100B
NO = 6                     # repairs per pass
GROUPS = 4                 # plane groups of 4 (15 combinations each)

# (k, r) shapes that get a generated kernel (the batched GF(2^16) shape of
# tools/bench_gf16.py and the tests)
GF16_BS_CONFIGS = [(64, 16), (16, 4), (32, 8)]


def mul(a: int, b: int) -> int:
    """GF(2^16) mod 0x1100B (gf_tables.rs:333-353 as intended)."""
    r = 0
    while b:
        if b & 1:
            r ^= a
        b >>= 1
        a <<= 1
        if a & 0x10000:
            a ^= POLY
    return r


@functools.lru_cache(maxsize=None)
def inv(a: int) -> int:
    if a == 0:
        raise ZeroDivisionError
    r, x, p = 1, a, 0xFFFE
    while p:
        if p & 1:
            r = mul(r, x)
        x = mul(x, x)
        p >>= 1
    return r


def cauchy16(k: int, r: int) -> list[list[int]]:
    """decoder.rs:77-80: C[j][i] = inv(i ^ (k + j))."""
    return [[inv(i ^ (k + j)) for i in range(k)] for j in range(r)]


def sigma(b: int) -> int:
    """Raw bit b of a loaded half-word -> symbol bit (big-endian symbols)."""
    return (b + 8) % 16


def raw_matrix(c: int) -> list[int]:
    """Row b (raw output plane) -> bit mask of raw input planes b'."""
    cols = [mul(c, 1 << u) for u in range(16)]     # column u: c * x^u
    rows = []
    for b in range(16):
        t = sigma(b)
        m = 0
        for bb in range(16):
            if (cols[sigma(bb)] >> t) & 1:
                m |= 1 << bb
        rows.append(m)
    return rows


def terms(k: int, r: int, p: int) -> list[list[list[tuple[int, int]]]]:
    """Pass p: terms[i][jj][b] = [(group, idx)] combination registers XORed
    into output plane b of repair 8p + jj for source row i."""
    C = cauchy16(k, r)
    out = []
    for i in range(k):
        per_j = []
        for jj in range(NO):
            j = NO * p + jj
            if j >= r:
                break
            rows = raw_matrix(C[j][i])
            per_j.append([[(g, (rows[b] >> (4 * g)) & 15) for g in range(GROUPS) if (rows[b] >> (4 * g)) & 15]
                          for b in range(16)])
        out.append(per_j)
    return out


def n_passes(r: int) -> int:
    return (r + NO - 1) // NO


# ---- CPU model of the schedule ---------------------------------------------

_TMASK = (0x55555555, 0x33333333, 0x0F0F0F0F, 0x00FF00FF)


def transpose16(x: np.ndarray) -> np.ndarray:
    """The 4-stage delta-swap network on 16 uint32 rows (axis 0), an
    involution: stage i swaps row bit i with column bit i."""
    x = x.copy()
    for i in range(4):
        s, m = 1 << i, np.uint32(_TMASK[i])
        for rr in range(16):
            if rr & s:
                continue
            a, b = x[rr], x[rr + s]
            t = ((a >> np.uint32(s)) ^ b) & m
            x[rr + s] = b ^ t
            x[rr] = a ^ (t << np.uint32(s))
    return x


def emulate(k: int, r: int, rows: np.ndarray) -> np.ndarray:
    """rows: (k, 64) uint8 = one lane's 4 units of each source row (any
    content).  Returns (r, 64) uint8: the lane's 4 units of each repair, by
    the generated kernels' schedule."""
    assert rows.shape == (k, 64)
    out = np.zeros((r, 64), np.uint8)
    for p in range(n_passes(r)):
        T = terms(k, r, p)
        nj = len(T[0])
        acc = np.zeros((nj, 16), np.uint32)
        for i in range(k):
            planes = transpose16(rows[i].view("<u4").copy())
            comb = {}
            for g in range(GROUPS):
                for idx in range(1, 16):
                    v = np.uint32(0)
                    for t in range(4):
                        if idx >> t & 1:
                            v ^= planes[4 * g + t]
                    comb[(g, idx)] = v
            for jj in range(nj):
                for b in range(16):
                    for ti in T[i][jj][b]:
                        acc[jj, b] ^= comb[ti]
        for jj in range(nj):
            out[NO * p + jj] = transpose16(acc[jj]).view(np.uint8)
    return out


# ---- C++ generation ----------------------------------------------------------

def _combo_stmts(needed: set[tuple[int, int]]) -> list[str]:
    """Statements defining c{g}_{idx} for the needed combinations (and the
    ones they are built from): singles are the planes themselves."""
    have: dict[tuple[int, int], str] = {}
    stmts = []

    def get(g: int, idx: int) -> str:
        if (g, idx) in have:
            return have[(g, idx)]
        bits = [t for t in range(4) if idx >> t & 1]
        if len(bits) == 1:
            have[(g, idx)] = f"x[{4 * g + bits[0]}]"
            return have[(g, idx)]
        hi = 1 << bits[-1]
        a = get(g, idx ^ hi)
        b = get(g, hi)
        name = f"c{g}_{idx}"
        stmts.append(f"const uint32_t {name} = bs_xor({a}, {b});")
        have[(g, idx)] = name
        return name

    for g, idx in sorted(needed):
        get(g, idx)
    return stmts, have


def _acc_stmt(acc: str, ops: list[str], init: bool) -> str:
    """acc (^)= XOR of ops with explicit v_xor3 / v_xor (opaque to the
    compiler: no reassociation, no re-splitting)."""
    if init:
        if not ops:
            return f"{acc} = 0u;"
        if len(ops) == 1:
            return f"{acc} = {ops[0]};"
        if len(ops) == 2:
            return f"{acc} = bs_xor({ops[0]}, {ops[1]});"
        return f"{acc} = bs_xor3({ops[0]}, {ops[1]}, {ops[2]});" + (
            f" {acc} = bs_xor({acc}, {ops[3]});" if len(ops) == 4 else "")
    if not ops:
        return ""
    if len(ops) == 1:
        return f"{acc} = bs_xor({acc}, {ops[0]});"
    return f"{acc} = bs_xor3({acc}, {ops[0]}, {ops[1]});"


def kernel_name(k: int, r: int, mode: str = "enc") -> str:
    return f"qf_gf16bs_k{k}_r{r}" if mode == "enc" else f"qf_gf16bs_{mode}_k{k}_r{r}"


def generate(k: int, r: int, mode: str = "enc") -> str:
    """One kernel per (k, r) holding every pass: block b runs pass
    (b / 8) % P over lane-chunk block ((b / 8) / P) * 8 + b % 8, so the P
    blocks that read the same rows share an XCD (blocks are dealt round-robin
    over the 8 XCDs) and run at about the same time: the re-reads of the
    later passes hit L2 instead of HBM.

    mode "syn" (decode syndromes, Decoder16 with Cauchy rows): source row i
    is gathered through the generation's slot map (a zero row where source i
    was not received), and repair j's output, if repair k + j was accepted at
    position a, is XORed with that repair row and stored as syndrome a."""
    P = n_passes(r)
    syn = mode == "syn"
    name = kernel_name(k, r, mode)
    lines = [f"// generated by quicfuscate_amd/gf16_codegen.py for k = {k}, r = {r}, {mode} -- do not edit",
             f"__global__ void __launch_bounds__(256, 2) {name}(Gf16BsArgs a) {{",
             f"    const uint32_t y = blockIdx.x >> 3, pass = y % {P}u;",
             f"    const uint64_t f = (uint64_t)((y / {P}u) * 8u + (blockIdx.x & 7u)) * 256u + threadIdx.x;",
             "    if (f >= a.total) return;",
             "    const Gf16BsLane ln = gf16bs_lane(a, f);"]
    if syn:
        lines.append("    if (a.skip[ln.g]) return;    // failed, nothing erased, or a repair the kernel has no row for")
        lines.append("    const uint16_t* sm = a.smap + ln.g * a.smap_gs;")
    lines += ["    uint32_t tm[4];",
              "    gf16bs_masks(tm);"]

    def load(i: int, indent: str) -> str:
        if syn:
            return f"{indent}gf16bs_load_row_sel(a, ln, sl{i}, nx);"
        return f"{indent}gf16bs_load_row(a, ln, {i}, nx);"

    for p in range(P):
        T = terms(k, r, p)
        nj = len(T[0])
        lines.append(f"    if (pass == {p}u) {{")
        lines.append("        uint32_t " + ", ".join(f"a{jj}_{b}" for jj in range(nj) for b in range(16)) + ";")
        lines.append("        uint32_t x[16], nx[16];")
        if syn:
            lines.append("        uint32_t sl0 = sm[0]" + (", sl1 = sm[1]" if k > 1 else "")
                         + "".join(f", sl{i}" for i in range(2, k)) + ";")
        lines.append(load(0, "        "))
        for i in range(k):
            lines.append("        {")
            lines.append("#pragma unroll")
            lines.append("            for (int d = 0; d < 16; ++d) x[d] = nx[d];")
            if i + 1 < k:
                if syn and i + 2 < k:
                    lines.append(f"            sl{i + 2} = sm[{i + 2}];")
                lines.append(load(i + 1, "            "))
            lines.append("            gf16bs_transpose(x, tm);")
            # groups {0, 1} then {2, 3}: 22 combinations live at a time, one
            # v_xor3 per output plane and group pair
            for half, gs in enumerate(((0, 1), (2, 3))):
                needed = {t for jj in range(nj) for b in range(16) for t in T[i][jj][b] if t[0] in gs}
                stmts, have = _combo_stmts(needed)
                lines.append("            {")
                lines += ["                " + s for s in stmts]
                for jj in range(nj):
                    for b in range(16):
                        ops = [have[t] for t in T[i][jj][b] if t[0] in gs]
                        lines.append("                " + _acc_stmt(f"a{jj}_{b}", ops, i == 0 and half == 0))
                lines.append("            }")
            # the accumulators through an empty asm: XOR chains are not
            # reassociated across rows (that would keep many rows' combinations
            # live at once)
            for jj in range(nj):
                ops = ", ".join(f'"+v"(a{jj}_{b})' for b in range(16))
                lines.append(f'            asm volatile("" : {ops});')
            lines.append("        }")
        for jj in range(nj):
            lines.append("        {")
            lines.append("            uint32_t o[16] = {" + ", ".join(f"a{jj}_{b}" for b in range(16)) + "};")
            lines.append("            gf16bs_transpose(o, tm);")
            store = "gf16bs_store_syn" if syn else "gf16bs_store_row"
            lines.append(f"            {store}(a, ln, {NO * p + jj}u, o);")
            lines.append("        }")
        lines.append("    }")
    lines.append("}")
    lines.append("")
    return "\n".join(lines)


def generate_all(configs=None) -> str:
    configs = configs or GF16_BS_CONFIGS
    body = [generate(k, r, m) for k, r in configs for m in ("enc", "syn")]
    table = ["static const Gf16BsEntry kGf16BsTable[] = {"]
    for k, r in configs:
        e, y = kernel_name(k, r), kernel_name(k, r, "syn")
        table.append(f'    {{{k}u, {r}u, {n_passes(r)}u, {e}, "{e}", {y}, "{y}"}},')
    table.append("};")
    return "\n".join(body + table) + "\n"
