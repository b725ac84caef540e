#!/usr/bin/env python3
"""VGPR-indexed XOR micro-benchmark (gfx950): the product step a bit-sliced
combine with wave-uniform runtime coefficients needs,

    acc_p ^= lo[i_p];  acc_p ^= hi[j_p]      (i_p, j_p in SGPRs)

as s_set_gpr_idx_on / s_set_gpr_idx_idx + v_xor_b32 with an M0-indexed src0,
against the same 16 XORs with fixed registers.  Checks the indexed results.

    python tools/ubench_idx.py build     # here: tools/lab_build/idx_*.hsaco
    python tools/ubench_idx.py run       # GPU box"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
OUT = REPO / "tools" / "lab_build"
LO, HI, ACC = 40, 56, 20


def body(kind: str) -> list[str]:
    ops = []
    if kind == "idx":
        for p in range(8):
            ops.append(f"s_set_gpr_idx_on s{8 + 2 * p}, gpr_idx(SRC0)" if p == 0 else f"s_set_gpr_idx_idx s{8 + 2 * p}")
            ops.append(f"v_xor_b32_e32 v{ACC + p}, v{LO}, v{ACC + p}")
            ops.append(f"s_set_gpr_idx_idx s{9 + 2 * p}")
            ops.append(f"v_xor_b32_e32 v{ACC + p}, v{HI}, v{ACC + p}")
        ops.append("s_set_gpr_idx_off")
    elif kind == "plain":
        for p in range(8):
            ops.append(f"v_xor_b32_e32 v{ACC + p}, v{LO + p}, v{ACC + p}")
            ops.append(f"v_xor_b32_e32 v{ACC + p}, v{HI + 15 - p}, v{ACC + p}")
    elif kind == "bitop3_banks":   # acc, LO, HI operands in three different VGPR banks
        for p in range(8):
            lo = LO + ((1 - (ACC + p)) % 4)          # bank (acc + 1) mod 4 ... chosen below
            ops.append(f"v_bitop3_b32 v{ACC + 4 * p}, v{ACC + 4 * p}, v{LO + 1 + 4 * (p % 4)}, v{HI + 2 + 4 * (p % 3)} bitop3:0x96")
            ops.append(f"v_bitop3_b32 v{ACC + 4 * p + 1}, v{ACC + 4 * p + 1}, v{LO + 2 + 4 * (p % 3)}, v{HI + 3 + 4 * (p % 3)} bitop3:0x96")
    elif kind == "bitop3_same":   # LO and HI operands in the accumulator's bank
        for p in range(8):
            ops.append(f"v_bitop3_b32 v{ACC + 4 * p}, v{ACC + 4 * p}, v{LO + 4 * (p % 4)}, v{HI + 4 * (p % 3)} bitop3:0x96")
            ops.append(f"v_bitop3_b32 v{ACC + 4 * p + 1}, v{ACC + 4 * p + 1}, v{LO + 1 + 4 * (p % 3)}, v{HI + 1 + 4 * (p % 3)} bitop3:0x96")
    elif kind == "xor_banks":
        for p in range(8):
            ops.append(f"v_xor_b32_e32 v{ACC + 4 * p}, v{LO + 1 + 4 * (p % 4)}, v{ACC + 4 * p}")
            ops.append(f"v_xor_b32_e32 v{ACC + 4 * p + 1}, v{LO + 2 + 4 * (p % 3)}, v{ACC + 4 * p + 1}")
    elif kind == "perm_banks":
        for p in range(8):
            ops.append(f"v_perm_b32 v{ACC + 4 * p}, v{LO + 1 + 4 * (p % 4)}, v{HI + 2 + 4 * (p % 3)}, v{ACC + 4 * p + 3}")
            ops.append(f"v_perm_b32 v{ACC + 4 * p + 1}, v{LO + 2 + 4 * (p % 3)}, v{HI + 3 + 4 * (p % 3)}, v{ACC + 4 * p + 3}")
    elif kind == "bitsel_sgpr":   # the transpose's bit-select: mask in an SGPR
        for p in range(8):
            ops.append(f"v_bitop3_b32 v{ACC + 4 * p}, s30, v{LO + 1 + 4 * (p % 4)}, v{HI + 2 + 4 * (p % 3)} bitop3:0xca")
            ops.append(f"v_bitop3_b32 v{ACC + 4 * p + 1}, s30, v{LO + 2 + 4 * (p % 3)}, v{HI + 3 + 4 * (p % 3)} bitop3:0xca")
    elif kind == "bitsel_vgpr":   # the same bit-select with the mask in a VGPR (v31)
        for p in range(8):
            ops.append(f"v_bitop3_b32 v{ACC + 4 * p}, v63, v{LO + 1 + 4 * (p % 4)}, v{HI + 2 + 4 * (p % 3)} bitop3:0xca")
            ops.append(f"v_bitop3_b32 v{ACC + 4 * p + 1}, v63, v{LO + 2 + 4 * (p % 3)}, v{HI + 3 + 4 * (p % 3)} bitop3:0xca")
    elif kind == "xor3_sgpr":   # 3-input XOR with one SGPR operand
        for p in range(8):
            ops.append(f"v_bitop3_b32 v{ACC + 4 * p}, s30, v{LO + 1 + 4 * (p % 4)}, v{HI + 2 + 4 * (p % 3)} bitop3:0x96")
            ops.append(f"v_bitop3_b32 v{ACC + 4 * p + 1}, s30, v{LO + 2 + 4 * (p % 3)}, v{HI + 3 + 4 * (p % 3)} bitop3:0x96")
    elif kind == "bitsel_vgpr_last":   # mask VGPR as the last operand (truth table 0xd8)
        for p in range(8):
            ops.append(f"v_bitop3_b32 v{ACC + 4 * p}, v{LO + 1 + 4 * (p % 4)}, v{HI + 2 + 4 * (p % 3)}, v63 bitop3:0xd8")
            ops.append(f"v_bitop3_b32 v{ACC + 4 * p + 1}, v{LO + 2 + 4 * (p % 3)}, v{HI + 3 + 4 * (p % 3)}, v63 bitop3:0xd8")
    elif kind in ("jump_xor3", "jump_xor3_noidx"):
        # one product per call: acc_j[p] ^= LO[a_p(c)] ^ HI[b_p(c)] for p < 8 in
        # the coefficient's code block (JUMP_BLOCK bytes at .Ltab + c * 128),
        # acc_j chosen by gpr_idx (DST, SRC0) = 8 j; 8 products per body
        for i, c in enumerate(JUMP_CS):
            if kind == "jump_xor3":
                ops.append(f"s_set_gpr_idx_idx s{24 + (i % 2)}")
            ops.append(f"s_add_u32 s42, s40, s{8 + i}")
            ops.append("s_addc_u32 s43, s41, 0")
            ops.append("s_swappc_b64 s[44:45], s[42:43]")
    elif kind == "plain_salu":   # same SALU count as idx, no indexing
        for p in range(8):
            ops.append(f"s_mov_b32 s{40 + 2 * p}, s{8 + 2 * p}")
            ops.append(f"v_xor_b32_e32 v{ACC + p}, v{LO + p}, v{ACC + p}")
            ops.append(f"s_mov_b32 s{41 + 2 * p}, s{9 + 2 * p}")
            ops.append(f"v_xor_b32_e32 v{ACC + p}, v{HI + 15 - p}, v{ACC + p}")
    return ops


JUMP_CS = (3, 77, 140, 201, 18, 255, 96, 5)    # the body's coefficients, in order


def jump_ab(c: int, p: int) -> tuple[int, int]:
    """The LO / HI table entries plane p of coefficient c's block reads
    (arbitrary but distinct per plane: the check recomputes them)."""
    return (c + 5 * p) & 15, (3 * c + p) & 15


def jump_table(kind: str) -> list[str]:
    """256 blocks of 128 B: 8 v_bitop3 (xor3) and the return."""
    lines = ["s_endpgm", ".p2align 7", ".Ltab:"]
    for c in range(256):
        for p in range(8):
            a, b = jump_ab(c, p)
            lines.append(f"v_bitop3_b32 v{ACC + p}, v{ACC + p}, v{LO + a}, v{HI + b} bitop3:0x96")
        lines.append("s_setpc_b64 s[44:45]")
        lines.append(".p2align 7")
    return lines


def kernel(name: str, kind: str, unroll: int = 4) -> str:
    lines = [
        "s_load_dwordx2 s[4:5], s[0:1], 0x0",
        "s_load_dword s6, s[0:1], 0x8",
        "v_and_b32_e32 v1, 63, v0",
        "v_lshlrev_b32_e32 v2, 4, v1",          # 16 lane
    ]
    for p in range(32):
        lines.append(f"v_mov_b32_e32 v{ACC + p}, 0")
    for i in range(16):
        lines.append(f"v_add_u32_e32 v{LO + i}, {i}, v2")
        lines.append(f"v_lshlrev_b32_e32 v{HI + i}, 16, v{LO + i}")
    lines.append("s_mov_b32 s30, 0x0f0f0f0f")
    lines.append("v_mov_b32_e32 v63, s30")
    jump = kind.startswith("jump")
    if jump:   # block offsets of the body's coefficients; the table's address; gpr_idx 0 / 8
        for i, c in enumerate(JUMP_CS):
            lines.append(f"s_mov_b32 s{8 + i}, {c * 128}")
        lines += ["s_getpc_b64 s[40:41]", ".Lpc:", "s_add_u32 s40, s40, .Ltab-.Lpc", "s_addc_u32 s41, s41, 0",
                  "s_mov_b32 s24, 0", "s_mov_b32 s25, 8"]
        if kind == "jump_xor3":
            lines.append("s_set_gpr_idx_on s24, gpr_idx(SRC0,DST)")
    else:
        for p in range(8):
            lines.append(f"s_mov_b32 s{8 + 2 * p}, {p}")
            lines.append(f"s_mov_b32 s{9 + 2 * p}, {15 - p}")
    lines.append("s_waitcnt lgkmcnt(0)")
    lines.append(".Lloop:")
    for _ in range(unroll):
        lines += body(kind)
    lines += ["s_sub_u32 s6, s6, 1", "s_cmp_lg_u32 s6, 0", "s_cbranch_scc1 .Lloop"]
    if kind == "jump_xor3":
        lines.append("s_set_gpr_idx_off")
    # out + (workgroup * 256 + tid) * 32 (jump kinds: * 64, two accumulator sets)
    sh = 6 if jump else 5
    lines += [f"s_lshl_b32 s7, s2, {sh + 8}", f"v_lshlrev_b32_e32 v4, {sh}, v0", "v_add_u32_e32 v4, s7, v4",
              "v_mov_b32_e32 v5, 0",
              "v_lshl_add_u64 v[10:11], v[4:5], 0, s[4:5]",
              f"global_store_dwordx4 v[10:11], v[{ACC}:{ACC + 3}], off",
              f"global_store_dwordx4 v[10:11], v[{ACC + 4}:{ACC + 7}], off offset:16"]
    if jump:   # the second accumulator set (gpr_idx 8) after the first
        lines += [f"global_store_dwordx4 v[10:11], v[{ACC + 8}:{ACC + 11}], off offset:32",
                  f"global_store_dwordx4 v[10:11], v[{ACC + 12}:{ACC + 15}], off offset:48"]
        lines += jump_table(kind)
    else:
        lines.append("s_endpgm")
    body_s = "\n".join("\t" + x if not x.endswith(":") else x for x in lines)
    for lbl in (".Lloop", ".Ltab", ".Lpc"):
        body_s = body_s.replace(lbl, f".L{name}_{lbl[2:]}")
    return f"""\t.amdgcn_target "amdgcn-amd-amdhsa--gfx950"
\t.amdhsa_code_object_version 6
\t.text
\t.globl\t{name}
\t.p2align\t8
\t.type\t{name},@function
{name}:
{body_s}
\t.section\t.rodata,"a",@progbits
\t.p2align\t6, 0x0
\t.amdhsa_kernel {name}
\t\t.amdhsa_kernarg_size 16
\t\t.amdhsa_user_sgpr_count 2
\t\t.amdhsa_user_sgpr_kernarg_segment_ptr 1
\t\t.amdhsa_system_sgpr_workgroup_id_x 1
\t\t.amdhsa_system_vgpr_workitem_id 0
\t\t.amdhsa_next_free_vgpr 128
\t\t.amdhsa_next_free_sgpr 64
\t\t.amdhsa_accum_offset 128
\t\t.amdhsa_reserve_vcc 0
\t.end_amdhsa_kernel
\t.text
.Lfunc_end_{name}:
\t.size\t{name}, .Lfunc_end_{name}-{name}
\t.amdgpu_metadata
---
amdhsa.kernels:
  - .args:
      - .address_space:  global
        .name:           out
        .offset:         0
        .size:           8
        .value_kind:     global_buffer
      - .name:           iters
        .offset:         8
        .size:           4
        .value_kind:     by_value
    .group_segment_fixed_size: 0
    .kernarg_segment_align: 8
    .kernarg_segment_size: 16
    .max_flat_workgroup_size: 256
    .name:           {name}
    .private_segment_fixed_size: 0
    .sgpr_count:     70
    .sgpr_spill_count: 0
    .symbol:         {name}.kd
    .vgpr_count:     128
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


KINDS = ["idx", "plain", "plain_salu", "bitop3_banks", "bitop3_same", "xor_banks", "perm_banks", "bitsel_sgpr",
         "bitsel_vgpr", "xor3_sgpr", "bitsel_vgpr_last", "jump_xor3", "jump_xor3_noidx"]


def valu_per_body(kind: str) -> int:
    return 8 * len(JUMP_CS) if kind.startswith("jump") else len([o for o in body(kind) if o.startswith("v_")])


def jump_expected(kind: str, lanes: np.ndarray) -> np.ndarray:
    """(lanes, 16) accumulators after one body of a jump kind (HI[7] is v63,
    which the prologue sets to the 0x0f0f0f0f mask after the tables)."""
    want = np.zeros((len(lanes), 16), np.uint32)
    for i, c in enumerate(JUMP_CS):
        j = (i % 2) if kind == "jump_xor3" else 0
        for p in range(8):
            a, b = jump_ab(c, p)
            hi = np.full(len(lanes), 0x0F0F0F0F, np.int64) if HI + b == 63 else (lanes * 16 + b) << 16
            want[:, 8 * j + p] ^= ((lanes * 16 + a) ^ hi).astype(np.uint32)
    return want


def build():
    from quicfuscate_amd.build_lib import assemble
    OUT.mkdir(parents=True, exist_ok=True)
    for k in KINDS:
        print(k, assemble(f"idx_{k}", kernel(f"idx_{k}", k), OUT))


def run(out):
    import torch
    hip = ctypes.CDLL(str(Path(torch.__file__).parent / "lib" / "libamdhip64.so"))
    stream = torch.cuda.current_stream()
    res = {}
    for k in KINDS:
        mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
        data = (OUT / f"idx_{k}.hsaco").read_bytes()
        buf = ctypes.create_string_buffer(data, len(data))
        assert hip.hipModuleLoadData(ctypes.byref(mod), buf) == 0
        assert hip.hipModuleGetFunction(ctypes.byref(fn), mod, f"idx_{k}".encode()) == 0
        for waves_per_simd in (1, 2, 4):
            blocks = 256 * waves_per_simd
            o = torch.zeros(blocks * 256 * (16 if k.startswith("jump") else 8), dtype=torch.int32, device="cuda")

            def launch(iters):
                ka = np.zeros(4, np.uint32)
                ka[0], ka[1], ka[2] = o.data_ptr() & 0xFFFFFFFF, o.data_ptr() >> 32, iters
                kb = ctypes.create_string_buffer(ka.tobytes(), 16)
                size = ctypes.c_size_t(16)
                extra = (ctypes.c_void_p * 5)(1, ctypes.cast(kb, ctypes.c_void_p), 2,
                                             ctypes.cast(ctypes.pointer(size), ctypes.c_void_p), 3)
                assert hip.hipModuleLaunchKernel(fn, blocks, 1, 1, 256, 1, 1, 0,
                                                 ctypes.c_void_p(stream.cuda_stream), None, extra) == 0
            launch(1)   # unroll 4: acc = 4 x the body = 0 -> use 1 iteration with odd unroll check below
            torch.cuda.synchronize()
            iters = 20000
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record(stream)
            launch(iters)
            t1.record(stream)
            torch.cuda.synchronize()
            ms = t0.elapsed_time(t1)
            waves = blocks * 4
            xors = waves * iters * 4 * valu_per_body(k)
            res[f"{k}@{waves_per_simd}w"] = {"ms": round(ms, 3),
                                             "xor_per_simd_per_ns": round(xors / 1024 / (ms * 1e6), 3)}
            print(k, waves_per_simd, res[f"{k}@{waves_per_simd}w"], flush=True)
        hip.hipModuleUnload(mod)
    # correctness of the indexed reads: a build with unroll 1, one iteration
    from quicfuscate_amd.build_lib import assemble
    h = (OUT / "idx_check.hsaco")
    mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
    data = h.read_bytes()
    buf = ctypes.create_string_buffer(data, len(data))
    assert hip.hipModuleLoadData(ctypes.byref(mod), buf) == 0
    assert hip.hipModuleGetFunction(ctypes.byref(fn), mod, b"idx_check") == 0
    o = torch.zeros(256 * 8, dtype=torch.int32, device="cuda")
    ka = np.zeros(4, np.uint32)
    ka[0], ka[1], ka[2] = o.data_ptr() & 0xFFFFFFFF, o.data_ptr() >> 32, 1
    kb = ctypes.create_string_buffer(ka.tobytes(), 16)
    size = ctypes.c_size_t(16)
    extra = (ctypes.c_void_p * 5)(1, ctypes.cast(kb, ctypes.c_void_p), 2,
                                 ctypes.cast(ctypes.pointer(size), ctypes.c_void_p), 3)
    assert hip.hipModuleLaunchKernel(fn, 1, 1, 1, 256, 1, 1, 0, ctypes.c_void_p(stream.cuda_stream), None, extra) == 0
    torch.cuda.synchronize()
    got = o.cpu().numpy().view(np.uint32).reshape(256, 8)
    lane = np.arange(256) % 64
    want = np.stack([(lane * 16 + p) ^ ((lane * 16 + 15 - p) << 16) for p in range(8)], axis=1).astype(np.uint32)
    res["idx_correct"] = bool((got == want).all())
    print("idx correct:", res["idx_correct"], flush=True)
    hip.hipModuleUnload(mod)
    for k in ("jump_xor3", "jump_xor3_noidx"):   # one body, one iteration
        mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
        data = (OUT / f"idx_check_{k}.hsaco").read_bytes()
        buf = ctypes.create_string_buffer(data, len(data))
        assert hip.hipModuleLoadData(ctypes.byref(mod), buf) == 0
        assert hip.hipModuleGetFunction(ctypes.byref(fn), mod, f"idx_check_{k}".encode()) == 0
        o = torch.zeros(256 * 16, dtype=torch.int32, device="cuda")
        ka[0], ka[1], ka[2] = o.data_ptr() & 0xFFFFFFFF, o.data_ptr() >> 32, 1
        kb = ctypes.create_string_buffer(ka.tobytes(), 16)
        extra = (ctypes.c_void_p * 5)(1, ctypes.cast(kb, ctypes.c_void_p), 2,
                                     ctypes.cast(ctypes.pointer(size), ctypes.c_void_p), 3)
        assert hip.hipModuleLaunchKernel(fn, 1, 1, 1, 256, 1, 1, 0, ctypes.c_void_p(stream.cuda_stream), None,
                                         extra) == 0
        torch.cuda.synchronize()
        got = o.cpu().numpy().view(np.uint32).reshape(256, 16)
        res[f"{k}_correct"] = bool((got == jump_expected(k, lane)).all())
        print(k, "correct:", res[f"{k}_correct"], flush=True)
        hip.hipModuleUnload(mod)
    Path(out).parent.mkdir(exist_ok=True)
    Path(out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["build", "run"])
    ap.add_argument("--out", default="gpurun_out/ubench_idx.json")
    a = ap.parse_args()
    if a.cmd == "build":
        build()
        from quicfuscate_amd.build_lib import assemble
        print(assemble("idx_check", kernel("idx_check", "idx", unroll=1), OUT))
        for k in ("jump_xor3", "jump_xor3_noidx"):
            print(assemble(f"idx_check_{k}", kernel(f"idx_check_{k}", k, unroll=1), OUT))
    else:
        run(a.out)
