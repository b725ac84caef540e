"""Build libqf_fec.so (gfx950) in-tree.

    python -m quicfuscate_amd.build_lib

Compiles quicfuscate_amd/csrc/*.hip with hipcc for gfx950 and links the
shared library against the HIP runtime that ships with PyTorch (same soname
as /opt/rocm's, so a process that imports torch holds exactly one HIP
runtime).  The asm-pipelined kernels keep in-flight load destinations in
registers; a register spill would copy them before the data lands, so the
build fails if any k_combine_* kernel reports scratch usage.
"""
from __future__ import annotations

import concurrent.futures as cf
import json
import os
import re
import shutil
import subprocess
import sys
import zlib
from pathlib import Path

PKG = Path(__file__).resolve().parent
REPO = PKG.parent
CSRC = PKG / "csrc"
OUT_DIR = PKG / "lib"
LIB = OUT_DIR / "libqf_fec.so"
LIB_ROCM = OUT_DIR / "libqf_fec_rocm.so"
SOURCES = ["qf_kernels.hip", "qf_api.hip", "qf_objects.hip", "qf_bs.hip", "qf_adaptive.hip", "qf_wire.hip",
           "qf_gf16.hip", "qf_objects16.hip", "qf_wiedemann.hip", "qf_gf16_bs.hip",
           "qf_gf16_fft.hip"]
# (k, r) Cauchy configurations that get a bit-sliced assembly kernel
# (bs_codegen.py); every other shape runs the general v_perm kernel.
BS_CONFIGS = [(64, 16), (64, 10), (32, 16), (16, 16), (16, 1), (32, 5), (48, 8), (96, 15)]
# C5 adaptive shapes (Normal/Medium windows, r = ceil(k * ratio) - k):
# r <= 16 above (encode, syndrome and fused decode kernels); larger r encode
# only, in passes
BS_ENC_ONLY = [(128, 20), (128, 39), (160, 48), (196, 59)]   # (128, 39): Medium default window
BS_PASS = 22   # repairs per pass: 8 r accumulator VGPRs, r <= 22 fits 256 at pd 3
# additive-FFT encode ('E', lch_fft.py): power-of-two k where the plan costs
# fewer plane ops than one coefficient block per repair
BS_FFT = [(64, 16), (64, 10), (32, 16), (16, 16)]
# additive-FFT encode passes of the C5 codes with more than 22 repairs
# (lch_fft.hybrid_plan: one pass per coset of 16 repair points, sources
# [0, 2^a) through the FFT, the rest folded in directly), merged ('N')
BS_FFT_PASSES = [(128, 20), (128, 39), (160, 48), (196, 59)]
# pass-major FFT synw ('Y') where its passes that run at 20 % loss cost less
# than the plain ones (tools/gpu_r04_c5y.sh, profiles/r04al_c5_hybrid_chunks.json:
# block decode (128, 39) 1,470 -> 1,784 GiB/s, (160, 48) 1,536 -> 1,700;
# (196, 59) 1,383 -> 1,262: three FFT passes run against two plain ones)
BS_FFT_SYNW = [(128, 39), (160, 48)]
BS_FFT_SYNW_SHARED = [(128, 20), (128, 39), (160, 48), (196, 59)]
BS_XCHG_EARLY = 3     # rows of the next group a shared-row wave loads before its transform
BS_FFT_DEC_HYBRID = [(96, 15), (48, 8)]   # fused FFT decode ('C') of C5 shapes with k not a power of two
BS_SLIDING_PLAIN = [(32, 5), (16, 1)]   # sliding-window encoders ('g'): plain pass, cached row loads
BS_SLIDING_FFT = [(48, 8)]              # ... hybrid FFT pass, cached row loads
BS_FFT_ENC_HYBRID = [(96, 15)]   # hybrid-plan FFT encode ('E'): sliding windows +35 %, block equal
BS_FFT_CH = 8
BS_FFT_DEC_PD = 2
BS_PD = 3
# gfx950 (CDNA4) only: the generated kernels are gfx950 assembly, and the
# HIP kernels assume its 160 KB of LDS per CU (k_decode_prepare_lu_lanes
# stages 72 KB statically, above the 64 KiB of gfx942 / gfx90a)
ARCH = "gfx950"


def _check_arch() -> None:
    """QF_OFFLOAD_ARCH may only name gfx950: checked where code is compiled or
    assembled, so importing this module (kernel_specs() in the CPU emulator
    tests) works whatever another project set that variable to."""
    arch = os.environ.get("QF_OFFLOAD_ARCH", "gfx950")
    if arch != "gfx950":
        raise RuntimeError(f"QF_OFFLOAD_ARCH={arch}: this library targets gfx950 (MI355X) only")


def _hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libqf_fec.so)")


def _clangxx() -> str:
    for cand in ("/opt/rocm/llvm/bin/clang++", shutil.which("clang++")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("clang++ not found")


def _torch_hip_runtime() -> Path:
    import importlib.util

    spec = importlib.util.find_spec("torch")
    if spec is None or spec.origin is None:
        raise RuntimeError("torch is required (its HIP runtime is the one linked)")
    lib = Path(spec.origin).parent / "lib" / "libamdhip64.so"
    if not lib.exists():
        raise RuntimeError(f"{lib} missing: need a ROCm build of torch")
    return lib


def _rocm_hip_runtime() -> Path:
    rocm = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
    lib = rocm / "lib" / "libamdhip64.so"
    if not lib.exists():
        raise RuntimeError(f"{lib} missing (ROCm HIP runtime)")
    return lib


def _compile(src: str, build_dir: Path, extra: list[str]) -> tuple[Path, str]:
    _check_arch()
    obj = build_dir / (Path(src).stem + ".o")
    cmd = [
        _hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
        "-Wno-unused-value", "-Wno-unused-result",
        f"-I{REPO / 'include'}", f"-I{CSRC}", f"-I{build_dir}",
        "-c", str(CSRC / src), "-o", str(obj),
    ] + extra
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{res.stderr[-4000:]}")
    return obj, res.stderr


def _check_no_scratch(remarks: str) -> dict[str, dict[str, int]]:
    usage: dict[str, dict[str, int]] = {}
    cur = None
    for line in remarks.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            usage[cur] = {}
            continue
        m = re.search(r"(VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+)", line)
        if m and cur:
            usage[cur][m.group(1).split(" ")[0]] = int(m.group(2))
    bad = [n for n, u in usage.items() if "combine" in n and u.get("ScratchSize", 0) > 0]
    if bad:
        raise RuntimeError(f"register spill in asm-pipelined kernels (unsafe): {bad}")
    return usage


def _check_gf16_bs(remarks: str) -> None:
    """The generated GF(2^16) kernels must keep their accumulators in
    registers: spilling them in the row loop would cost more than the kernel
    saves (gf16_codegen.py).  A few spilled VGPRs (k = 64: 8, the output
    pointers, stored once before the rows and reloaded for the stores) are
    allowed."""
    usage = _check_no_scratch(remarks)
    bad = {n: u for n, u in usage.items() if "gf16bs" in n and u.get("VGPRs", 0) > 256}
    spills = re.findall(r"VGPRs Spill: (\d+)", remarks)
    if bad or any(int(x) > 16 for x in spills):
        raise RuntimeError(f"gf16 bit-sliced kernels spill VGPRs: {bad or spills}")


def assemble(name: str, asm_text: str, out_dir: Path) -> Path:
    """gfx950 assembly text -> code object (.hsaco) via clang + ld.lld."""
    _check_arch()
    clang = _clangxx().replace("clang++", "clang")
    lld = str(Path(clang).parent / "ld.lld")
    asm = out_dir / f"{name}.s"
    asm.write_text(asm_text)
    obj = asm.with_suffix(".o")
    hsaco = asm.with_suffix(".hsaco")
    res = subprocess.run([clang, "-x", "assembler", "-target", "amdgcn-amd-amdhsa", f"-mcpu={ARCH}",
                          "-c", str(asm), "-o", str(obj)], capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"assembling {asm.name} failed:\n{res.stderr[-3000:]}")
    res = subprocess.run([lld, "-shared", str(obj), "-o", str(hsaco)], capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"linking {asm.name} failed:\n{res.stderr[-3000:]}")
    return hsaco


def kernel_specs() -> list:
    """Every generated kernel the library embeds (bs_codegen.KernelSpec), in
    table order."""
    from . import bs_codegen as bs
    from . import lch_fft

    specs = [bs.KernelSpec(k, r, BS_PD, mode) for mode in ("enc", "syn", "dec") for (k, r) in BS_CONFIGS]
    # fused decode over the lane-chunk layout (one generation per lane; the
    # default decode, 'c'); the 'd' kernels above stay for QF_DECODE_LEGACY=1
    specs += [bs.KernelSpec(k, r, BS_PD, "dec", chunked=True) for (k, r) in BS_CONFIGS]
    # small batches ('k'): the four waves of a workgroup split one item's rows
    specs += [bs.KernelSpec(k, r, BS_PD, "dec", chunked=True, ksplit=4) for (k, r) in BS_CONFIGS]
    for k, rt in BS_ENC_ONLY:
        npass = -(-rt // BS_PASS)   # balanced passes (each pass re-reads the sources)
        j0 = 0
        for p in range(npass):
            rp = (rt - j0) // (npass - p)
            specs.append(bs.KernelSpec(k, rp, BS_PD, "enc", r_total=rt, j0=j0))
            # small batches ('f'): the four waves of a workgroup split one item's sources
            specs.append(bs.KernelSpec(k, rp, BS_PD, "enc", r_total=rt, j0=j0, ksplit=4))
            j0 += rp
    # decode syndromes of the same codes for long rows (slot map read by the
    # scalar unit, _generate_synw): same balanced passes, items whose
    # generations accepted no repair of a pass skip it
    for k, rt in BS_ENC_ONLY:
        npass = -(-rt // BS_PASS)
        j0 = 0
        for p in range(npass):
            rp = (rt - j0) // (npass - p)
            specs.append(bs.KernelSpec(k, rp, BS_PD, "synw", r_total=rt, j0=j0))
            j0 += rp
    # additive-FFT encode ('E'): default cache policy for the row loads (the
    # boundary line a 1,200-B row shares with the next row / the neighbouring
    # item stays in L2; non-temporal loads re-fetch it: FETCH_SIZE 1.085x ->
    # 1.019x the source bytes, 1.133 -> 1.114 ms, profiles/r04a_lab_enc_traffic.json)
    specs += [bs.KernelSpec(k, r, BS_PD, "enc", fft=BS_FFT_CH, ld_policy="") for (k, r) in BS_FFT]
    # (one hybrid pass for (96, 15) / (48, 8), whose repair points share one
    # coset of 16: 19.5 k -> 16.2 k VALU per item at (96, 15), but block encode
    # 4,703 -> 4,450 / 5,024 -> 4,841 GiB/s against sliding 758 -> 831 /
    # 1,232 -> 1,325; not in the library, profiles/r04an_c5_single_hybrid.json)
    # (round 5, natural coset fill: 12.6 k VALU per item at (96, 15), and the
    # block encode no slower, profiles/r05bi_c5_single_pass_fft.json; in the
    # library block 4,807-4,844 against 4,799-4,819 GiB/s, sliding windows, whose
    # overlapping rows come from cache, 1,023-1,033 against 754-764; (48, 8):
    # block 4,862-4,868 against 4,994-5,007, sliding 1,273 against 1,179-1,223,
    # a wash, so it stays plain; profiles/r05bk_c5_hybrid_encode.json)
    specs += [bs.KernelSpec(k, r, BS_PD, "enc", fft=BS_FFT_CH, ld_policy="") for (k, r) in BS_FFT_ENC_HYBRID]
    # sliding windows ('g', QF_SLIDING_KERNELS: chosen when the generations of a
    # batch overlap, generation stride < k row strides): consecutive windows
    # share k - 1 rows, so the row loads keep the default cache policy (the
    # block encoders' non-temporal loads drop the rows the next window reads),
    # and (48, 8) takes the hybrid FFT pass that was a wash for block encode
    # but not for windows (1,273 against 1,179-1,223 GiB/s, round 5)
    specs += [bs.KernelSpec(k, r, BS_PD, "enc", ld_policy="", sliding=True) for (k, r) in BS_SLIDING_PLAIN]
    specs += [bs.KernelSpec(k, r, BS_PD, "enc", fft=BS_FFT_CH, ld_policy="", sliding=True)
              for (k, r) in BS_SLIDING_FFT]
    # additive-FFT fused decode ('C'): pd 2 (the ring holds a chunk + pd rows)
    # (default cache policy: neighbouring 1,200-B rows share their boundary
    # lines, and non-temporal loads / stores drop them before the reuse;
    # tools/dec_lab.py, profiles/r03_lab_dec_policy.json: 1.485 -> 1.39 ms)
    # (round 4: interleaved LU products and 64-bit-shift transposes /
    # selectors: 1.409 -> 1.358-1.364 ms, profiles/r04d_lab_dec_ilp_s64.json)
    # (round 5: non-temporal recovered-row stores, loads still at the default
    # policy: 1.357-1.387 -> 1.345-1.352 ms, profiles/r05_lab_dec.json r05k)
    # (round 5: also the C5 shapes whose k is not a power of two, through the
    # hybrid plan: (96, 15) 30.4 k -> 22.4 k VALU per item, its 7-quad slot map
    # run as a window; (48, 8) 10.6 k -> 9.4 k)
    specs += [bs.KernelSpec(k, r, BS_FFT_DEC_PD, "dec", chunked=True, fft=BS_FFT_CH, ld_policy="", st_policy="nt",
                            early_stores=True, lu_ilp=True, bfi_transpose="s64")
              for (k, r) in BS_FFT + BS_FFT_DEC_HYBRID]
    # ((32, 5) with chunks of 4 rows, 160 VGPRs and 5.1 k VALU per item against
    # the plain kernel's 152 and 5.5 k, measured 2-4 % slower: block decode
    # 4,227-4,242 against 4,305-4,402 GiB/s, profiles/r05ap_c5_fft_decode_ch4.json)
    # every pass of a C5 code in one dispatch ('M' plain, 'N' additive-FFT
    # passes; QF_ENCODE_MERGED): one wave per pass on the workgroup's item, so
    # the source rows come from HBM once.  Plain passes: 4 waves where 3 would
    # leave a quarter of a CU's 8 wave slots (2 per SIMD at > 128 VGPRs) empty
    for k, rt in BS_ENC_ONLY:
        npass = -(-rt // BS_PASS)
        if npass == 1:
            continue
        npass += npass == 3
        cuts = [rt * p // npass for p in range(npass + 1)]
        specs.append(bs.merged_spec([bs.KernelSpec(k, cuts[p + 1] - cuts[p], BS_PD, "enc", r_total=rt, j0=cuts[p])
                                     for p in range(npass)]))
    # (tools/gpu_r04_c5fft.sh, profiles/r04v_c5_passes.json: 1,508 -> 1,962 GiB/s
    # at (160, 48), 1,347 -> 1,552 at (196, 59), 2,371 -> 2,600 at (128, 39);
    # (128, 20) keeps its single plain pass: 4,568 against 3,806 merged FFT)
    # (round 5: the passes' waves share loads, transposes and chunk butterflies
    # through LDS, xchg: 0.506-0.541 -> 0.323-0.325 ms at (196, 59), 0.446 ->
    # 0.320 at (160, 48), 0.438 -> 0.304 at (128, 39), bit-exact,
    # tools/c5_lab.py, profiles/r05u_c5_xchg.json)
    # (a code of 3 passes gets a producer-only 4th wave, so two workgroups fill a
    # CU's 8 wave slots and a round holds 4 groups: 0.322-0.333 -> 0.305 ms at
    # (160, 48), 0.309-0.316 -> 0.299-0.302 at (128, 39), profiles/r05ae_c5_helper.json)
    # (each wave issues the loads of its next group's first 3 rows before
    # transforming the current group, xchg_early: 0.315-0.329 -> 0.305-0.316 ms
    # at (196, 59), tools/c5_lab.py, profiles/r05au_c5_xchg_early.json)
    # ((128, 20), two coset passes of 16 + 4: shared-row FFT passes 0.231-0.235
    # ms against 0.241-0.250 for its single plain pass on the same box; with
    # two producer-only waves 0.272-0.278, so none; tools/c5_lab.py,
    # profiles/r05bg_c5_128_20.json)
    for k, rt in BS_FFT_PASSES:
        cps = lch_fft.coset_passes(k, rt)
        three = len(cps) >= 3
        specs.append(bs.merged_spec([bs.KernelSpec(k, rp, BS_PD, "enc", fft=BS_FFT_CH, ld_policy="", r_total=rt, j0=j0,
                                                   xchg_early=BS_XCHG_EARLY if three else 0)
                                     for j0, rp in cps], xchg=True, helpers=1 if len(cps) == 3 else 0))
    # the synw passes of the C5 codes in one pass-major dispatch: one launch
    # of P x n workgroups instead of P launches of n, so a pass's last, partly
    # filled round overlaps the next pass's first; 'Y' the additive-FFT passes
    # (one per coset of 16 repair points, as the 'N' encode; QF_FFT_KERNELS),
    # 'X' the plain ones
    for k, rt in BS_FFT_SYNW:
        specs.append(bs.merged_spec([bs.KernelSpec(k, rp, BS_PD, "synw", fft=BS_FFT_CH, ld_policy="", r_total=rt,
                                                   j0=j0) for j0, rp in lch_fft.coset_passes(k, rt)], concat=True))
    # the FFT synw passes item-major, their waves sharing the row gather,
    # transposes and chunk butterflies through LDS ('Z', QF_SYNW_SHARED; the
    # sources are read once instead of once per pass)
    # (a producer-only 4th wave, as the encode's, measured no faster here: (160, 48) block
    # decode 2,007-2,019 against 2,025-2,031 GiB/s, profiles/r05af_c5_helper_decode.json)
    for k, rt in BS_FFT_SYNW_SHARED:
        cps = lch_fft.coset_passes(k, rt)
        specs.append(bs.merged_spec([bs.KernelSpec(k, rp, BS_PD, "synw", fft=BS_FFT_CH, ld_policy="", r_total=rt,
                                                   j0=j0, xchg_early=BS_XCHG_EARLY if len(cps) >= 3 else 0)
                                     for j0, rp in cps], xchg=True))
    for k, rt in BS_ENC_ONLY:
        npass = -(-rt // BS_PASS)
        if npass == 1:
            continue
        j0, passes = 0, []
        for p in range(npass):
            rp = (rt - j0) // (npass - p)
            passes.append(bs.KernelSpec(k, rp, BS_PD, "synw", r_total=rt, j0=j0))
            j0 += rp
        specs.append(bs.merged_spec(passes, concat=True))
    # (the synw passes merged item-major -- bs_codegen.merged_spec takes
    # them -- measured no faster: 0.479 / 0.546 / 0.467 ms against 0.485 /
    # 0.529 / 0.482 at (160, 48) / (196, 59) / (128, 39), profiles/r04z_c5_merged.json;
    # those passes are not bound by their row reads)
    # bit-sliced payload pass with wave-uniform runtime coefficients ('m')
    # (cmb_lean: the gpr_idx mode on for a row's whole product run, the early
    # exit every 4 outputs: 2.47 -> 2.40 ms at e = 39, 1.34 -> 1.27-1.29 for the
    # wide pass at e = 20, tools/cmb_lab.py, profiles/r05az_cmb_lab.json; rows
    # two ahead (cmb_pf2) measured neutral, profiles/r05ba_cmb_lab.json)
    specs.append(bs.KernelSpec(0, 16, BS_PD, "cmb", cmb_lean=True))
    # ... and every pass of it in one pass-major launch ('P', QF_ENCODE_MERGED)
    specs.append(bs.KernelSpec(0, 16, BS_PD, "cmb", pass_major=True, cmb_lean=True))
    # ... and its item-major interleave ('Q', QF_COMBINE_XCD): the passes of
    # one slot on one XCD at once, the later passes' syndrome reads from L2
    specs.append(bs.KernelSpec(0, 16, BS_PD, "cmb", pass_major=True, cmb_lean=True, pm_xcd=True))
    # ... and the wide single pass for 17-24 outputs (QF_COMBINE_WIDE): each
    # input row read and transposed once instead of once per pass
    # (e = 20: 1.60 -> 1.34 ms, tools/cmb_lab.py, profiles/r05ay_cmb_lab.json)
    specs.append(bs.KernelSpec(0, bs.CMB_WIDE_R, BS_PD, "cmb", cmb_lean=True))
    # ... and all four with the products as calls into per-coefficient code
    # blocks (QF_COMBINE_JUMP: 'j' single / wide, 'J' pass-major, 'V'
    # interleaved): e = 39, 3 passes 2.41-2.53 -> 2.17 ms, e = 16 1.14 -> 1.00
    # (tools/cmb_lab.py, profiles/r06j_cmb_lab.json)
    specs.append(bs.KernelSpec(0, 16, BS_PD, "cmb", cmb_lean=True, cmb_jump=3))
    specs.append(bs.KernelSpec(0, bs.CMB_WIDE_R, BS_PD, "cmb", cmb_lean=True, cmb_jump=3))
    specs.append(bs.KernelSpec(0, 16, BS_PD, "cmb", pass_major=True, cmb_lean=True, cmb_jump=3))
    specs.append(bs.KernelSpec(0, 16, BS_PD, "cmb", pass_major=True, cmb_lean=True, pm_xcd=True, cmb_jump=3))
    # ... and 24-output passes in one pass-major launch ('W', QF_COMBINE_PM24):
    # e_max 33-48 in 2 passes instead of 3, 49-72 in 3 instead of 4
    specs.append(bs.KernelSpec(0, bs.CMB_WIDE_R, BS_PD, "cmb", pass_major=True, cmb_lean=True, cmb_jump=3))
    return specs


def bs_codegen_wide() -> int:
    from . import bs_codegen as bs
    return bs.CMB_WIDE_R


def _cmb_mode(spec) -> str:
    """Table letter of a payload-pass kernel (qf_bs.hip cmb_entry): 'm' / 'P' /
    'Q' (single or wide / pass-major / interleaved), 'j' / 'J' / 'V' the same
    with jump-table products; 'W' the 24-output pass-major passes (jump)."""
    if spec.pass_major and spec.r == bs_codegen_wide():
        return "W"
    if spec.pass_major:
        return ("V" if spec.cmb_jump else "Q") if spec.pm_xcd else ("J" if spec.cmb_jump else "P")
    return "j" if spec.cmb_jump else "m"


def _bs_kernels(build_dir: Path) -> Path:
    """Generate + assemble the bit-sliced kernels; emit a C include that
    embeds the code objects, and lib/kernel_hashes.json (sha256 of every code
    object by kernel name: profiles/ record the hash of the kernel they
    measured, bench.py uses a profile's counters only while it matches)."""
    import hashlib

    from . import bs_codegen as bs

    entries, blobs = [], []
    specs = kernel_specs()
    hashes = {}
    for n, spec in enumerate(specs):
        k, r = spec.k, spec.r
        hsaco = assemble(spec.name, bs.emit_asm(spec, bs.generate(spec)), build_dir)
        data = hsaco.read_bytes()
        hashes[spec.name] = hashlib.sha256(data).hexdigest()[:16]
        # zlib-compressed (about 3x smaller; qf_bs.hip inflates a code object
        # once, on its first load): the library is pushed to the GPU box on
        # every call, and these objects are most of its bytes
        z = zlib.compress(data, 9)
        hexs = ",".join(str(b) for b in z)
        blobs.append(f"static const unsigned char qf_bs_blob_{n}[] = {{{hexs}}};")
        if isinstance(spec, bs.MergedSpec):
            if spec.mode == "synw":
                mode = ("Z" if spec.passes[0].xchg else "Y") if spec.fft else "X"
            else:
                mode = "N" if spec.fft else "M"
        elif getattr(spec, "sliding", False):
            mode = "g"
        elif spec.chunked:
            mode = "C" if spec.fft else "k" if spec.ksplit > 1 else "c"
        elif spec.fft:
            mode = "E"
        elif spec.mode == "enc" and spec.ksplit > 1:
            mode = "f"
        else:
            mode = {"enc": "e", "syn": "s", "dec": "d", "synw": "w", "cmb": _cmb_mode(spec)}[spec.mode]
        entries.append(f"    {{{k}u, {r}u, {spec.pd}u, {spec.rt}u, {spec.j0}u, '{mode}', {spec.map_stride}u, \"{spec.name}\", "
                       f"qf_bs_blob_{n}, {len(data)}u, {getattr(spec, 'waves', 4)}u, "
                       f"{getattr(spec, 'n_passes', 1)}u, sizeof(qf_bs_blob_{n})}},")
    # the loader caches one module per table entry (qf_bs.h BsCache::kMax)
    kmax = int(re.search(r"kMax = (\d+)", (CSRC / "qf_bs.h").read_text()).group(1))
    if len(specs) > kmax:
        raise RuntimeError(f"{len(specs)} generated kernels > BsCache::kMax = {kmax} (qf_bs.h)")
    OUT_DIR.mkdir(exist_ok=True)
    (OUT_DIR / "kernel_hashes.json").write_text(json.dumps(hashes, indent=0, sort_keys=True))
    inc = build_dir / "qf_bs_blobs.inc"
    inc.write_text("// generated by quicfuscate_amd/build_lib.py from bs_codegen.py -- do not edit\n"
                   + "\n".join(blobs) + "\nstatic const QfBsEntry qf_bs_table[] = {\n"
                   + "\n".join(entries) + "\n};\n")
    return inc


def build(verbose: bool = False) -> Path:
    build_dir = PKG / "build"
    build_dir.mkdir(exist_ok=True)
    OUT_DIR.mkdir(exist_ok=True)
    _bs_kernels(build_dir)
    # bit-sliced GF(2^16) Cauchy encode kernels (HIP C++, gf16_codegen.py)
    from . import gf16_codegen
    inc16 = build_dir / "qf_gf16_bs.inc"
    text16 = gf16_codegen.generate_all()
    if not inc16.exists() or inc16.read_text() != text16:
        inc16.write_text(text16)
    with cf.ThreadPoolExecutor(max_workers=4) as ex:
        futs = {
            s: ex.submit(_compile, s, build_dir,
                         ["-Rpass-analysis=kernel-resource-usage"] if s in ("qf_kernels.hip", "qf_gf16_bs.hip")
                         else [])
            for s in SOURCES
        }
        objs = []
        for s in SOURCES:
            obj, err = futs[s].result()
            objs.append(obj)
            if s == "qf_gf16_bs.hip":
                _check_gf16_bs(err)
            if s == "qf_kernels.hip":
                usage = _check_no_scratch(err)
                if verbose:
                    for n, u in sorted(usage.items()):
                        print(f"  {n}: {u}")
    # two links of the same objects: libqf_fec.so against torch's HIP runtime
    # (the Python harness, one runtime per process) and libqf_fec_rocm.so
    # against /opt/rocm's (a host with no torch: the C-ABI caller, a Rust
    # binding -- INTEGRATION.md)
    for lib, hip in ((LIB, _torch_hip_runtime()), (LIB_ROCM, _rocm_hip_runtime())):
        tmp = lib.with_suffix(".so.tmp")
        cmd = [_clangxx(), "-shared", "-o", str(tmp)] + [str(o) for o in objs] + [
            str(hip), f"-Wl,-rpath,{hip.parent}", "-Wl,--no-undefined", "-lstdc++", "-lz",
        ]
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"link failed:\n{res.stderr[-4000:]}")
        os.replace(tmp, lib)
    return LIB


if __name__ == "__main__":
    p = build(verbose="-v" in sys.argv)
    print(p)
