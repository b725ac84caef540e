"""Generate tests/golden/golden16.json -- golden vectors for the GF(2^16)
"Extreme" codec.

Independent pure-Python restatement (no code shared with oracle/qf_oracle16.c):

  * gf_tables.rs:333-353  gf16_mul, shift-and-add mod 0x1100B (the reduction
                          the code intends; as written the u16 test of bit 16
                          never fires and does not compile)
  * gf_tables.rs:355-376  gf16_inv = x^(65534)
  * decoder.rs:77-80      Cauchy coefficients inv((i as u16) ^ ((k + j) as u16))
  * decoder.rs:21-75      repair = XOR over the window of c_i * s_i on
                          big-endian u16 symbols, j + 1 < len
  * decoder.rs:563-640    first k rows, Gauss-Jordan with pivot search, payloads
                          carried for systematic rows too (F4 fix)

Inputs: the reference test's own fixture (tests/fec.rs:52-82 gf16_encode_decode:
make_packet payloads of 8 bytes of value i % 255, k = 8, n = 12, packet 0
dropped) and the synthetic (7i + 13t + 1) & 255 pattern of SURVEY 8(c).

    python tests/golden/gen_golden16.py     # rewrites golden16.json
"""
from __future__ import annotations

import hashlib
import json
from pathlib import Path

OUT = Path(__file__).resolve().parent / "golden16.json"


def mul(a: int, b: int) -> int:
    res = 0
    while b:
        if b & 1:
            res ^= a
        b >>= 1
        a <<= 1
        if a & 0x10000:
            a ^= 0x1100B
    return res


def inv(a: int) -> int:
    if a == 0:
        raise ZeroDivisionError("gf16_inv(0) panics in the reference")
    r, x, p = 1, a, 0x10000 - 2
    while p:
        if p & 1:
            r = mul(r, x)
        x = mul(x, x)
        p >>= 1
    return r


def cauchy16(k: int, r: int) -> list[list[int]]:
    return [[inv((i & 0xFFFF) ^ ((k + j) & 0xFFFF)) for i in range(k)] for j in range(r)]


def encode16(src: list[bytes], r: int, L: int) -> list[bytes]:
    k = len(src)
    C = cauchy16(k, r)
    out = []
    for j in range(r):
        rep = bytearray(L)
        for i in range(k):
            c = C[j][i]
            for t in range(0, L - 1, 2):
                s = src[i][t] << 8 | src[i][t + 1]
                v = mul(c, s) ^ (rep[t] << 8 | rep[t + 1])
                rep[t], rep[t + 1] = v >> 8, v & 0xFF
        out.append(bytes(rep))
    return out


def decode16(k: int, row_index: list[int], rows: list[bytes], L: int) -> list[bytes]:
    rows = rows[:k]
    row_index = row_index[:k]
    m, pay = [], []
    for idx, data in zip(row_index, rows):
        if idx < k:
            m.append([1 if c == idx else 0 for c in range(k)])
        else:
            m.append([inv((i & 0xFFFF) ^ (idx & 0xFFFF)) for i in range(k)])
        pay.append([data[t] << 8 | data[t + 1] for t in range(0, L - 1, 2)])
    for i in range(k):
        p = next(q for q in range(i, k) if m[q][i])
        m[i], m[p] = m[p], m[i]
        pay[i], pay[p] = pay[p], pay[i]
        iv = inv(m[i][i])
        m[i] = [mul(x, iv) for x in m[i]]
        pay[i] = [mul(x, iv) for x in pay[i]]
        for q in range(k):
            f = m[q][i]
            if q != i and f:
                m[q] = [a ^ mul(f, b) for a, b in zip(m[q], m[i])]
                pay[q] = [a ^ mul(f, b) for a, b in zip(pay[q], pay[i])]
    return [bytes(b for v in row for b in (v >> 8, v & 0xFF)) for row in pay]


def h(chunks) -> str:
    d = hashlib.sha256()
    for c in chunks:
        d.update(bytes(c))
    return d.hexdigest()[:32]


def main() -> None:
    g: dict = {}
    g["mul"] = [[a, b, mul(a, b)] for a, b in ((0x8000, 2), (2, 0x8000), (0x1234, 0x5678), (0xFFFF, 0xFFFF),
                                               (0x100B, 0x100B), (1, 0xBEEF), (0, 7))]
    g["inv"] = [[a, inv(a)] for a in (1, 2, 3, 0x1234, 0x8000, 0xFFFF)]
    C = cauchy16(8, 4)
    g["cauchy_k8_r4"] = C
    g["cauchy_k64_r16_sha"] = h(v.to_bytes(2, "big") for row in cauchy16(64, 16) for v in row)
    g["cauchy_k1024_r8_row0_head"] = cauchy16(1024, 8)[0][:8]
    # tests/fec.rs:52-82: make_packet(i, i % 255) -> 8 bytes; k = 8, n = 12
    k, n, L = 8, 12, 8
    src = [bytes([i % 255] * L) for i in range(k)]
    reps = encode16(src, n - k, L)
    g["fec_rs_gf16_repairs"] = [list(x) for x in reps]
    arrival = list(range(1, k)) + [k + j for j in range(n - k)]
    rows = [src[a] if a < k else reps[a - k] for a in arrival]
    sol = decode16(k, arrival, rows, L)
    assert all(sol[i] == src[i] for i in range(k))
    g["fec_rs_gf16_decoded_first_bytes"] = [s[0] for s in sol]
    # SURVEY 8(c) synthetic pattern
    for k, r, L in ((16, 16, 1200), (64, 16, 1200)):
        src = [bytes(((7 * i + 13 * t + 1) & 255) for t in range(L)) for i in range(k)]
        g[f"encode16_k{k}_r{r}_L{L}_sha"] = h(encode16(src, r, L))
    OUT.write_text(json.dumps(g, indent=1) + "\n")


if __name__ == "__main__":
    main()
