#!/usr/bin/env python3
"""bench.py -- GF(256) RLNC encode+decode throughput on MI355X (device resident).

One "step" = one batched systematic Cauchy encode of G generations
(k=64 sources, r=16 repairs, 1200-byte packets) followed by one
batched decode of the same G generations at 20 % source loss (exactly 13
erased sources per generation, surviving sources then repairs in arrival
order, first-k-rows rule).  Inputs are resident in HBM before
the timed region.  value = source payload bytes of all ranks / max-over-
ranks step time, in GiB/s.

  python bench.py                          # N=1
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Multi-GPU: independent generations, each rank encodes/decodes its own G
(weak scaling, no collective on the data path); RCCL (torch 'nccl') only
carries the barrier, the max-over-ranks time and the verification counts.
"""
from __future__ import annotations

import argparse
import json
import os
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent
SEED = 0x51464543  # "QFEC"
PEAK_HBM_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def shard_generations(total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous generation range [lo, hi) of a rank."""
    lo = total * rank // world
    hi = total * (rank + 1) // world
    return lo, hi


def erasure_plan(G: int, k: int, e: int, seed: int) -> np.ndarray:
    """Seeded per-generation erasure sets (sorted source indices), shape (G, e)."""
    rng = np.random.default_rng(seed)
    keys = rng.random((G, k), dtype=np.float32)
    return np.sort(np.argsort(keys, axis=1)[:, :e], axis=1).astype(np.int64)


def arrival_index(erased: np.ndarray, k: int, r: int) -> np.ndarray:
    """Arrival order per generation: surviving sources ascending, then repairs."""
    G, e = erased.shape
    keep = np.ones((G, k), bool)
    np.put_along_axis(keep, erased, False, axis=1)
    surv = np.nonzero(keep)[1].reshape(G, k - e)
    reps = np.broadcast_to(np.arange(k, k + r), (G, r))
    return np.concatenate([surv, reps], axis=1).astype(np.uint16)


def payload_word_offset(rank: int, G: int, k: int, L: int) -> int:
    """splitmix64 word index of a rank's first source byte: every rank
    encodes distinct payload (the global generation index picks the words)."""
    return (rank * G * k * L) // 8


def _pg(dist, world: int) -> bool:
    """Collectives run when a process group exists: every N > 1 run, and the
    one-rank rehearsal of the RCCL branch (--force-pg)."""
    return world > 1 or (dist is not None and dist.is_available() and dist.is_initialized())


def reduce_max(torch, dist, values, world: int, device) -> list:
    """Max over ranks of [step_ms, enc_ms, dec_ms, failed] (the bench
    contract: the slowest rank defines the step time; any failure fails)."""
    t = torch.tensor(values, dtype=torch.float64, device=device)
    if _pg(dist, world):
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.tolist()


def xor_fold(torch, buf) -> int:
    """XOR of all 64-bit words of a device buffer (length % 8 == 0)."""
    w = buf.view(torch.int64)
    while w.numel() > 1:
        if w.numel() % 2:
            w = torch.cat([w, torch.zeros(1, dtype=torch.int64, device=w.device)])
        w = torch.bitwise_xor(w[0::2], w[1::2])
    return int(w.item()) & ((1 << 64) - 1)


def broadcast_descriptor(torch, dist, lib, k: int, r: int, Lb: int, G: int, e: int, world: int, device) -> bool:
    """rank 0 broadcasts the run descriptor and the r x k Cauchy
    coefficient matrix; every rank checks them against its own (the shards
    must encode the same code).  Returns this rank's match flag."""
    import ctypes

    mine = np.zeros(r * k, np.uint8)
    if lib.qf_cauchy_coeffs(k, r, mine.ctypes.data_as(ctypes.c_void_p)) != 0:
        return False
    d = torch.tensor([k, r, Lb, G, e, SEED], dtype=torch.int64, device=device)
    c = torch.from_numpy(mine.copy()).to(device)
    if _pg(dist, world):
        dist.broadcast(d, src=0)
        dist.broadcast(c, src=0)
    return d.tolist() == [k, r, Lb, G, e, SEED] and bool((c.cpu().numpy() == mine).all())


def gather_folds(torch, dist, fold: int, world: int, device) -> list:
    """Every rank's repair XOR-fold (RCCL all_gather: XOR is not a reduction op)."""
    t = torch.tensor([fold - (1 << 64) if fold >= 1 << 63 else fold], dtype=torch.int64, device=device)
    if not _pg(dist, world):
        return [fold]
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [int(x.item()) & ((1 << 64) - 1) for x in out]


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--G", type=int, default=None,
                    help="generations per GPU of the headline workload (default 65,536 = C2/C3 at every N; "
                         "156,250 = C4's 10 M packets/GPU with --config c4)")
    ap.add_argument("--config", choices=("auto", "c2c3", "c4"), default="auto",
                    help="auto / c2c3: C2+C3 per GPU at every N (weak scaling, identical per-GPU work); "
                         "c4: the headline runs C4's 156,250 generations per GPU")
    ap.add_argument("--c4-G", type=int, default=156250,
                    help="generations per rank of the separately timed C4 leg (10 M packets/GPU; 0 = skip)")
    ap.add_argument("--c4-steps", type=int, default=5)
    ap.add_argument("--c4-split", action="store_true",
                    help="C4 leg on the split-phase stream plan; default serial: at 156,250 generations the "
                         "encode's grid holds every CU until it drains, so the acceptance pass runs after it, "
                         "grid-capped (profiles/r03ab_c4_schedule.json)")
    ap.add_argument("--rank-sample", type=int, default=64,
                    help="seeded generations per rank checked against the CPU oracle (N>1 and --config c4)")
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--r", type=int, default=16)
    ap.add_argument("--L", type=int, default=1200)
    ap.add_argument("--erase", type=int, default=13, help="erased sources per generation (20%% of 64)")
    ap.add_argument("--cpu-sample", type=int, default=4096, help="generations in the CPU baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--c3b-G", type=int, default=65536,
                    help="generations of the C3 secondary variant (i.i.d. 20 %% loss over all k + r rows; 0 = skip)")
    ap.add_argument("--host-path-G", type=int, default=16384, help="generations for the pinned-host encode rate (0=skip)")
    ap.add_argument("--c5-mixed-bytes", type=float, default=4e9,
                    help="C5 (BASELINE configs[4]): source bytes of the heterogeneous batch; 0 skips the c5 leg")
    ap.add_argument("--c5-shape-bytes", type=float, default=1e9, help="C5: source bytes per shape and mode")
    ap.add_argument("--overlap", action="store_true",
                    help="run the step's encode and decode (independent batches) on two HIP streams")
    ap.add_argument("--split", action="store_true", default=True,
                    help="(default) decode acceptance pass on a 2nd stream beside the encode, payload pass after it")
    ap.add_argument("--serial", dest="split", action="store_false",
                    help="encode, then the whole decode, on one stream")
    ap.add_argument("--payload-stream", action="store_true", default=True,
                    help="(default) split, with the decode's payload pass enqueued on the encode's stream "
                         "(qf_ctx_set_payload_stream) instead of waiting for it across streams")
    ap.add_argument("--cross-stream", dest="payload_stream", action="store_false",
                    help="split, with the payload pass on the decode's stream waiting for the encode's event")
    ap.add_argument("--detail", default="gpurun_out/bench_detail.json",
                    help="file for the full per-leg record (the stdout line is the compact form, <= LINE_MAX bytes); "
                         "'' = do not write it")
    ap.add_argument("--stream-priority", action="store_true",
                    help="encode / payload stream at high HIP stream priority (split schedule)")
    ap.add_argument("--force-pg", action="store_true",
                    help="initialise the process group even at world size 1 (rehearses the RCCL branch on one GPU)")
    a = ap.parse_args(argv)
    if a.overlap:
        a.split = False
    return a


def cgroup_cpu_quota(root: str = "/sys/fs/cgroup"):
    """CPUs' worth of the cgroup's CPU quota (v2 cpu.max, else v1 cfs quota /
    period, floored, at least 1); None without a quota."""
    root = Path(root)
    try:
        q, per = (root / "cpu.max").read_text().split()[:2]
        if q != "max":
            return max(1, int(q) // int(per))
        return None
    except (OSError, ValueError):
        pass
    try:
        q = int((root / "cpu" / "cpu.cfs_quota_us").read_text())
        per = int((root / "cpu" / "cpu.cfs_period_us").read_text())
        return max(1, q // per) if q > 0 and per > 0 else None
    except (OSError, ValueError):
        return None


def launch_plan(args, env, argv=None):
    """--gpus N > 1 with no launcher in the environment (WORLD_SIZE unset): the
    command that starts N rank processes (torch.distributed.run on 127.0.0.1,
    one process per GPU), run as a child before this process touches the GPU.
    None when this process is a rank (or N == 1); an error string when the
    launcher's world size disagrees with --gpus."""
    import sys

    ws = env.get("WORLD_SIZE")
    if ws is None:
        if args.gpus <= 1:
            return None
        port = env.get("MASTER_PORT") or str(29500 + (os.getpid() % 2000))
        return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
                "--master-addr=127.0.0.1", f"--master-port={port}", str(Path(__file__).resolve())] + \
            list(sys.argv[1:] if argv is None else argv)
    if int(ws) != args.gpus:
        return f"WORLD_SIZE={ws} but --gpus {args.gpus}: refusing to report a line for the wrong GPU count"
    return None


def main(argv=None):
    args = parse(argv)
    plan = launch_plan(args, os.environ, argv)
    if isinstance(plan, str):
        import sys

        print(f"bench.py: {plan}", file=sys.stderr, flush=True)
        return 2
    if plan:
        import subprocess

        # the ranks run as children; this process never initialises the GPU
        return subprocess.call(plan)
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU over RCCL ("nccl"); QF_BENCH_BACKEND=gloo rehearses
    # the multi-rank path on fewer GPUs (ranks share devices round robin)
    backend = os.environ.get("QF_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    pg = world > 1 or args.force_pg
    if pg:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    from quicfuscate_amd import _lib as L
    from quicfuscate_amd import fec

    lib = L._lib()
    # the headline runs the same per-GPU work at every N (weak scaling); C4's
    # 10 M packets per GPU run as their own timed leg (c4_leg) unless the
    # headline itself is C4 (--config c4)
    c4 = args.config == "c4"
    if args.G is None:
        args.G = 156250 if c4 else 65536   # C4: 10,000,000 packets / 64 per generation
    k, r, Lb, G, e = args.k, args.r, args.L, args.G, args.erase
    dev = torch.device("cuda", local)
    desc_ok = broadcast_descriptor(torch, dist, lib, k, r, Lb, G, e, world, dev if backend == "nccl" else "cpu")
    # A dedicated stream for the library AND torch: torch's default stream is
    # handle 0, which the C ABI would replace by a private stream, and the
    # timing events must be recorded on the stream the kernels run on.
    # --stream-priority: the step's main stream (encode, then the payload pass)
    # at high priority, so the split acceptance pass on the decode's stream
    # only takes wave slots the encode leaves free
    stream = torch.cuda.Stream(dev, priority=-1 if args.stream_priority else 0)
    torch.cuda.set_stream(stream)
    ctx = fec.Context(local, stream.cuda_stream)

    # --- inputs (resident in HBM before timing) ---------------------------
    # Repair rows are blocks of Lr = round_up(L, 128) bytes that are zero
    # beyond L, as the reference's pool blocks (decoder.rs:182/264,
    # optimize.rs:524); QF_ENCODE_ZERO_TAIL lets the kernel write the tail, so
    # it stores whole 128-B lines.  Algorithmic bytes count L per row.
    Lr = (Lb + 127) // 128 * 128
    src = torch.empty(G * k * Lb, dtype=torch.uint8, device=dev)
    rep = torch.zeros(G * r * Lr, dtype=torch.uint8, device=dev)
    word_off = payload_word_offset(rank, G, k, Lb)
    L.check(lib.qf_fill_splitmix_dev(ctx.handle, src.data_ptr(), src.numel(), SEED, word_off), "fill")
    enc_args = dict(src_row_stride=Lb, src_gen_stride=k * Lb, rep_row_stride=Lr, rep_gen_stride=r * Lr, G=G,
                    zero_tail=True)
    fec.encode_batch(src, rep, k, r, Lb, ctx=ctx, **enc_args)

    erased = erasure_plan(G, k, e, SEED + rank)
    aidx = arrival_index(erased, k, r)
    n_slots = aidx.shape[1]
    rows = torch.empty(G * n_slots * Lb, dtype=torch.uint8, device=dev)
    srcv, repv, rowsv = src.view(G, k, Lb), rep.view(G, r, Lr)[:, :, :Lb], rows.view(G, n_slots, Lb)
    aidx_t = torch.from_numpy(aidx.astype(np.int64)).to(dev)
    CH = 4096
    for g0 in range(0, G, CH):
        g1 = min(G, g0 + CH)
        both = torch.cat([srcv[g0:g1], repv[g0:g1]], dim=1)
        gi = torch.arange(g1 - g0, device=dev)[:, None].expand(-1, n_slots)
        rowsv[g0:g1] = both[gi, aidx_t[g0:g1]]
        del both
    row_index = torch.from_numpy(aidx.view(np.int16)).to(dev)
    emax = min(k, r)
    rec = torch.empty(G * emax * Lb, dtype=torch.uint8, device=dev)
    rec_index = torch.empty(G * emax, dtype=torch.int16, device=dev)
    n_rec = torch.empty(G, dtype=torch.int32, device=dev)
    status = torch.empty(G, dtype=torch.int32, device=dev)
    dec_args = dict(max_rows=n_slots, row_stride=Lb, rows_gen_stride=n_slots * Lb, rec_row_stride=Lb,
                    rec_gen_stride=emax * Lb, G=G)

    # --overlap: the step's encode and decode work on different buffers (the
    # decode reads `rows`, built before timing; the encode writes `rep`), so
    # they can run on two streams forked from and joined back into `stream`:
    # the HBM-bound encode and the VALU-bound decode then share the CUs.
    #
    # --split: the encode stays on `stream`; the decode's acceptance pass
    # (row indices only) runs on a second stream beside the encode, and its
    # payload pass waits for the encode (qf_ctx_set_payload_wait), so the two
    # heavy kernels still run one after the other.
    if args.overlap:
        s_enc, s_dec = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
        ctx_enc, ctx_dec = fec.Context(local, s_enc.cuda_stream), fec.Context(local, s_dec.cuda_stream)
    elif args.split:
        s_enc, s_dec = stream, torch.cuda.Stream(dev)
        ctx_enc, ctx_dec = ctx, fec.Context(local, s_dec.cuda_stream)
    else:
        s_enc = s_dec = stream
        ctx_enc = ctx_dec = ctx
    ctxs = [ctx_enc] if ctx_enc is ctx_dec else [ctx_enc, ctx_dec]

    def encode():
        fec.encode_batch(src, rep, k, r, Lb, ctx=ctx_enc, **enc_args)

    def decode():
        fec.decode_batch(rows, row_index, rec, rec_index, n_rec, status, k, r, Lb, ctx=ctx_dec, **dec_args)

    def step(e0, e_enc, e_dec, e1):
        e0.record(stream)
        if args.overlap:
            s_enc.wait_event(e0)
            s_dec.wait_event(e0)
        if args.split:
            s_dec.wait_event(e0)
        encode()
        e_enc.record(s_enc)
        if args.split and args.payload_stream:
            ctx_dec.set_payload_stream(stream)     # payload pass after the encode, same stream
        elif args.split:
            ctx_dec.set_payload_wait(e_enc)
        decode()
        e_dec.record(stream if (args.split and args.payload_stream) else s_dec)
        if args.overlap:
            stream.wait_event(e_enc)
            stream.wait_event(e_dec)
        if args.split and not args.payload_stream:
            stream.wait_event(e_dec)
        e1.record(stream)

    def events():
        return tuple(torch.cuda.Event(enable_timing=True) for _ in range(4))

    for _ in range(args.warmup):
        step(*events())
    torch.cuda.synchronize()
    if _pg(dist, world):
        dist.barrier()
    torch.cuda.synchronize()

    ev = [events() for _ in range(args.steps)]
    for c in ctxs:
        c.profile(True)  # per-kernel HIP events on each launch stream
    t0 = time.perf_counter()
    for s in range(args.steps):
        step(*ev[s])
    torch.cuda.synchronize()
    if _pg(dist, world):
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ktimes = {}
    for c in ctxs:
        ktimes.update(c.kernel_times())
        c.profile(False)
    kern_ms = {n: ms / max(1, cnt) for n, (cnt, ms) in ktimes.items()}  # per launch
    kern_step_ms = {n: ms / args.steps for n, (cnt, ms) in ktimes.items()}
    # encode: step start -> encode done; decode: encode done (serial) or step
    # start (overlap) -> decode done
    enc_ms = float(np.mean([a.elapsed_time(b) for a, b, _, _ in ev]))
    dec_ms = float(np.mean([(a if args.overlap else b).elapsed_time(c) for a, b, c, _ in ev]))
    step_ms = wall * 1e3 / args.steps
    # with a second stream the encode shares the GPU with the decode's
    # acceptance pass (split) or the whole decode (overlap): its own roofline
    # comes from a few launches alone, after the timed steps (same buffers and
    # bytes; the repairs are rewritten with the same values)
    enc_alone_ms = None
    if ctx_enc is not ctx_dec:
        ctx_enc.profile(True)
        for _ in range(5):
            encode()
        ctx_enc.sync()
        ka = ctx_enc.kernel_times()
        ctx_enc.profile(False)
        ka = {n: ms / max(1, c) for n, (c, ms) in ka.items() if n.startswith(("qf_cauchy_bs", "k_combine_uniform"))}
        enc_alone_ms = next(iter(ka.values()), None)

    # --- verification (size-independent round trip on the device) ---------
    st_ok = bool((status == 0).all().item())
    n_ok = bool((n_rec == e).all().item())
    er_t = torch.from_numpy(erased).to(dev)
    idx_ok = bool((rec_index.view(G, emax)[:, :e].long() == er_t).all().item())
    recv = rec.view(G, emax, Lb)[:, :e]
    gi = torch.arange(G, device=dev)[:, None].expand(-1, e)
    bytes_ok = bool((recv == srcv[gi, er_t]).all().item())
    tails_zero = bool((rep.view(G, r, Lr)[:, :, Lb:] == 0).all().item())
    checksum = int(rep.view(torch.int64).sum().item()) & ((1 << 64) - 1)
    folds = gather_folds(torch, dist, xor_fold(torch, rep), world, dev if backend == "nccl" else "cpu")
    verified = st_ok and n_ok and idx_ok and bytes_ok and tails_zero

    coll_dev = dev if backend == "nccl" else "cpu"
    # C4: >= 64 seeded generations per rank against the CPU oracle
    sample_ok = None
    if c4 and args.rank_sample > 0:
        sample_ok = rank_oracle_sample(torch, src, rep, rows, aidx, rec, k, r, Lb, Lr, e, G, args.rank_sample,
                                       SEED + rank)
    sample_flags = gather_flags(torch, dist, -1 if sample_ok is None else int(sample_ok), world, coll_dev)
    desc_flags = gather_flags(torch, dist, int(desc_ok), world, coll_dev)
    step_ms_max, enc_ms_max, dec_ms_max, fails = reduce_max(
        torch, dist, [step_ms, enc_ms, dec_ms, 0.0 if (verified and sample_ok is not False and desc_ok) else 1.0], world,
        coll_dev)

    src_bytes_total = world * G * k * Lb
    gib = 1 << 30
    value = src_bytes_total / (step_ms_max / 1e3) / gib
    enc_gibps = src_bytes_total / (enc_ms_max / 1e3) / gib
    dec_gibps = src_bytes_total / (dec_ms_max / 1e3) / gib

    # Roofline of the dominant kernel (largest time per step), algorithmic
    # bytes per launch (DESIGN.md "Kernels"):
    #   encode (bit-sliced or v_perm): read k rows, write r rows / generation
    #   syndromes (decode stage A): read the k accepted rows + slot map,
    #     write e syndrome rows
    #   slots combine: stage B after syndromes (read e syndrome rows + e+1
    #     records, write e rows) or, on the general path, read k rows +
    #     records, write e rows
    #   prepare: row indices in, slot map / records / indices out
    #   fused decode: read the k accepted rows + slot map + LU record, write
    #     the e recovered rows
    fast_decode = any(n.startswith("qf_cauchy_syn") for n in ktimes)
    map_stride = (k + r + 15) // 16 * 16
    enc_bytes = G * (k + r) * Lb
    syn_bytes = G * ((k + e) * Lb + map_stride)
    dec_kernel_bytes = G * ((k + e) * Lb + map_stride + 272)
    if fast_decode:
        slots_bytes = G * (2 * e * Lb + (e + 1) * 16)
    else:
        slots_bytes = G * (k * Lb + e * Lb + (n_slots + 1) * 16)
    if any(n.startswith("qf_cauchy_dec") for n in ktimes):
        prep_bytes = G * (n_slots * 2 + map_stride + 272 + e * 2 + 8)   # row indices in; map, LU record out
    else:
        prep_bytes = G * (n_slots * 2 + map_stride + (r + 1) * 16 + e * 2 + 12)
    dec_bytes = G * (k * Lb + e * k + e * Lb)  # decode as a whole (SURVEY B_dec)

    def alg_bytes(name):
        if name.startswith("qf_cauchy_dec"):
            return dec_kernel_bytes
        if name.startswith("qf_cauchy_syn"):
            return syn_bytes
        if name.startswith("k_combine_slots"):
            return slots_bytes
        if name.startswith("k_decode_prepare"):
            return prep_bytes
        return enc_bytes

    dom = max(kern_step_ms, key=kern_step_ms.get)
    tfile = REPO / "profiles" / "traffic.json"
    sqfile = REPO / "profiles" / "sq_counters.json"
    hfile = REPO / "quicfuscate_amd" / "lib" / "kernel_hashes.json"
    try:
        code_sha = json.loads(hfile.read_text())
    except Exception:
        code_sha = {}

    def profile_current(name, ent):
        """A committed counter profile describes this run's kernel only if it
        recorded the code object it measured and the built kernel still has
        that hash (no stale counters in the line)."""
        want = next((v for n_, v in code_sha.items() if name == n_ or name.startswith(n_)), None)
        return want is not None and ent.get("code_sha16") == want
    props = torch.cuda.get_device_properties(dev)
    n_simd = 4 * props.multi_processor_count
    clk_ghz = (getattr(props, "clock_rate", 0) or 2_400_000) / 1e6   # kHz -> GHz (MI355X engine clock 2.4)

    def valu_roof(name, ms):
        """VALU issue of the kernel's launch: SQ_INSTS_VALU per wave x waves
        (rocprofv3 --pmc pass of this workload, profiles/sq_counters.json) at
        2 cycles per wave64 instruction per SIMD (MI355X_MICROARCH.md,
        per-instruction constants: wave64 VALU throughput 2 cyc on SIMD-32 with
        two or more waves; measured 0.95-1.03 wave-instructions per SIMD per ns,
        profiles/r02_ubench_idx.json), against the launch time measured here.
        A lower bound on issue time: half-rate ops (v_perm, 3-source ops with
        an SGPR operand) count one instruction."""
        try:
            sq = json.loads(sqfile.read_text())
        except Exception:
            return None
        ent = next((v for n_, v in sq.items() if n_ == name or n_.startswith(name)), None)
        if not ent or not ent.get("SQ_WAVES") or not profile_current(name, ent):
            return None
        per_wave = ent["SQ_INSTS_VALU"] / ent["SQ_WAVES"]
        waves = ent["SQ_WAVES"]
        issue_ms = per_wave * waves * 2 / (n_simd * clk_ghz * 1e9) * 1e3
        peak = n_simd * clk_ghz * 1e9 / 2 / 1e9          # wave-instructions per ns -> G/s
        # VALU lane-ops per GF byte multiply-add of the launch
        # (encode r k L G, decode e k L G byte-mult-adds)
        bm = (e if name.startswith("qf_cauchy_dec") else r) * k * Lb * G
        per_bm = round(per_wave * waves * 64 / bm, 4) if bm and not name.startswith("k_") else None
        return {"bound": "valu", "achieved": round(per_wave * waves / (ms / 1e3) / 1e9, 2), "peak": round(peak, 2),
                "lane_ops_per_byte_mult": per_bm,
                "unit": "G wave64 VALU instr/s", "frac": round(issue_ms / ms, 4),
                "valu_per_wave": round(per_wave, 1), "waves": int(waves), "issue_ms": round(issue_ms, 4),
                "source": "profiles/sq_counters.json (SQ_INSTS_VALU / SQ_WAVES, separate --pmc pass of this workload; "
                          "its code_sha16 equals the built kernel's)"}

    def roofline(name):
        ms = kern_ms[name]
        achieved = alg_bytes(name) / (ms / 1e3) / 1e9
        traffic = None
        if tfile.exists():
            try:
                tj = json.loads(tfile.read_text()).get(name, {})
                if (tj.get("k") == k and tj.get("r") == r and tj.get("L") == Lb and tj.get("G") == G
                        and profile_current(name, tj)):
                    traffic = tj.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        # the roof priced is HBM (byte work, no MFMA); what actually limits the
        # kernel comes from its SQ counters and the decode lab (DESIGN 3.2
        # "Round 5", profiles/r05_lab_dec.json): the fused decode's row loop
        # alone (no solve, no stores) reads at 6.06 TB/s in 0.83 ms; the
        # per-lane solve (half-rate v_perm products) and the recovered-row
        # stores add 0.55 ms, only partly hidden behind the partner wave's loads
        if name.startswith("qf_cauchy_dec"):
            limiter = "solve_issue_not_hidden"
        elif name.startswith(("k_combine", "k_decode_prepare")):
            limiter = "valu_issue"
        else:
            limiter = "hbm"
        vr = valu_roof(name, ms)
        if vr is not None and vr["frac"] > achieved / PEAK_HBM_GBPS:
            limiter = "valu_issue"
        return {"kernel": name, "launch_ms": round(ms, 4), "bound": "hbm", "limiter": limiter,
                "achieved": round(achieved, 1), "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                "frac": round(achieved / PEAK_HBM_GBPS, 4), "valu": vr, "traffic": traffic,
                "traffic_source": ("profiles/traffic.json: FETCH_SIZE x2 + WRITE_SIZE from separate rocprofv3 --pmc "
                                   "runs of this workload, not this run; the profile's code_sha16 equals the built "
                                   "kernel's (quicfuscate_amd/lib/kernel_hashes.json)" if traffic is not None else
                                   "none: no --pmc pass of the kernel as built (profiles/traffic.json code_sha16)"),
                "algorithmic_bytes_per_launch": alg_bytes(name)}

    enc_kernel = next((n for n in kern_ms if n.startswith(("qf_cauchy_bs", "k_combine_uniform"))), None)

    def roofline_encode():
        """The encode kernel's roofline: alone (5 launches after the timed
        steps) when the step runs it beside other work, with its in-step
        launches under `in_step`; the in-step figures otherwise."""
        rl = roofline(enc_kernel)
        if enc_alone_ms is None:
            return rl
        in_step = {key: rl[key] for key in ("launch_ms", "achieved", "frac")}
        rl["launch_ms"] = round(enc_alone_ms, 4)
        rl["achieved"] = round(alg_bytes(enc_kernel) / (enc_alone_ms / 1e3) / 1e9, 1)
        rl["frac"] = round(rl["achieved"] / PEAK_HBM_GBPS, 4)
        rl["valu"] = valu_roof(enc_kernel, enc_alone_ms)
        rl["timing"] = "the kernel alone: 5 launches on the context stream after the timed steps (HIP events)"
        rl["in_step"] = dict(in_step, note="its launches inside the timed steps, beside the decode's acceptance pass")
        return rl

    out = {
        "metric": "GF(256) RLNC encode+decode GiB/s device-resident, 1200B pkts gen=64, 1/2/4/8 GPU",
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_ms_max, 4),
        # the median of the per-step device times (HIP events
        # around each step on this rank) beside the wall-clock mean above
        "ms_per_step_median_rank0": round(float(np.median([a.elapsed_time(d) for a, _, _, d in ev])), 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (splitmix64 payload, seed 0x51464543; seeded 13-of-64 source erasures)",
        "config": {
            "workload": f"C2 encode + C3 decode: k={k}, r={r}, L={Lb}, G={G} generations/GPU, "
                        f"{e} erased sources/generation (20% loss), first-k-rows acceptance",
            "generations_per_gpu": G, "k": k, "r": r, "L": Lb, "erased": e,
            "parallelism": f"independent generations x{world} (weak)",
        },
        "encode_gibps": round(enc_gibps, 3),
        "decode_gibps": round(dec_gibps, 3),
        "encode_ms": round(enc_ms_max, 4),
        "decode_ms": round(dec_ms_max, 4),
        "decode_hbm_gbps": round(dec_bytes / (dec_ms / 1e3) / 1e9, 1),
        "kernel_ms_per_launch": {n: round(v, 4) for n, v in kern_ms.items()},
        "kernel_gbps": {n: round(alg_bytes(n) / (v / 1e3) / 1e9, 1) for n, v in kern_ms.items()},
        # dominant kernel (largest time per step); the fused decode is
        # VALU-issue-bound, its HBM fraction is reported as measured
        # (profiles/ SQ counters)
        "roofline": roofline(dom),
        # the encode kernel BASELINE.json's north star targets (>= 70 % HBM)
        "roofline_encode": roofline_encode() if enc_kernel else None,
        "streams": ("encode || decode (2 HIP streams)" if args.overlap else
                    ("encode, then decode payload pass on the same stream (qf_ctx_set_payload_stream); decode "
                     "acceptance pass on a 2nd stream beside the encode" if args.payload_stream else
                     "encode, then decode payload pass; decode acceptance pass on a 2nd stream beside the encode")
                    if args.split else "encode then decode (1 stream)"),
        "verified": bool(fails == 0),
        "repair_checksum_rank0": checksum,
        "repair_xor_fold_by_rank": [f"{f:016x}" for f in folds],
        "process_group": {"backend": dist.get_backend() if pg else None,
                          "world_size": dist.get_world_size() if pg else 1,
                          "env_world_size": world},
        "run_descriptor": {"broadcast_from_rank0": pg, "fields": ["k", "r", "L", "G", "erased", "seed"],
                           "cauchy_matrix_bytes": r * k, "matches_by_rank": [bool(f == 1) for f in desc_flags]},
    }
    if c4:
        out["config"]["workload"] = (f"C4 independent-generation encode + C3-shape decode sharded over {world} rank(s): "
                                     f"k={k}, r={r}, L={Lb}, G={G} generations/rank ({G * k:,} packets/rank), "
                                     f"{e} erased sources/generation")
        out["rank_oracle_sample"] = {"generations_per_rank": args.rank_sample,
                                     "pass_by_rank": [None if f < 0 else bool(f) for f in sample_flags]}
    if pg:
        out["sliding_halo"] = sliding_halo_leg(torch, dist, ctx, lib, L, rank, world, dev, backend)

    if rank == 0 and world == 1:
        out["hbm_copy_context"] = copy_bandwidth(torch)

    if rank == 0 and world == 1 and args.c3b_G > 0:
        out["c3_bernoulli"] = c3_bernoulli_leg(torch, fec, ctx, srcv, repv, k, r, Lb, min(args.c3b_G, G), dev)

    if rank == 0 and world == 1 and args.host_path_G > 0:
        out["host_path"] = host_path_rate(torch, lib, L, ctx, k, r, Lb, min(args.host_path_G, G))
        out["host_path"]["decode"] = host_decode_rate(torch, lib, L, ctx, rows, row_index, rec, e, n_slots, k, r,
                                                      Lb, min(args.host_path_G, G))

    if rank == 0 and world == 1 and not args.no_cpu:
        S = min(args.cpu_sample, G)
        rep_dense = repv[:S].contiguous().view(-1)
        out["cpu_host"] = cpu_host()
        out["cpu_baseline"] = cpu_baseline(src, rep_dense, rows, aidx, rec, n_rec, rec_index, k, r, Lb, e, S)
        out["cpu_variants"] = cpu_variants(src, rep_dense, k, r, Lb, S)
        out["cpu_c1"] = cpu_c1(torch, fec, ctx, Lb)
        out["cpu_gf_mul_loop"] = cpu_gf_mul_loop()

    if args.c4_G > 0 and not c4:
        # free the headline's buffers (about 13 GB) before C4's (about 31 GB per rank)
        del src, rep, rows, rowsv, srcv, repv, rec, rec_index, n_rec, status, aidx_t, row_index, er_t, recv, gi
        torch.cuda.empty_cache()
        out["c4"] = c4_leg(torch, dist, fec, L, lib, ctx, stream, dev, rank, world, backend, k, r, Lb, e, args.c4_G,
                           args.c4_steps, args.warmup, args.rank_sample, split=args.c4_split)

    if rank == 0 and world == 1 and args.c5_mixed_bytes > 0:
        out["c5"] = c5_leg(fec, ctx, args.c5_mixed_bytes, args.c5_shape_bytes)

    if rank == 0:
        detail = emit_detail(out, args.detail)
        print(json.dumps(compact_line(out, detail)), flush=True)
    if pg:
        dist.destroy_process_group()
    if args.split:
        ctx_dec.close()
    if args.overlap:
        ctx_enc.close()
        ctx_dec.close()
    ctx.close()


def c4_leg(torch, dist, fec, L, lib, ctx, stream, dev, rank, world, backend, k, r, Lb, e, G, steps, warmup,
           rank_sample, split=False) -> dict:
    """BASELINE C4: 10 M packets = 156,250 generations per rank,
    encoded and then decoded at the C3 loss shape (13 erased sources per
    generation), each rank on its own contiguous generations with distinct
    payload; timed like the headline (barrier + synchronize around the steps,
    max over ranks); every recovered byte and zero tail checked on the device,
    plus seeded generations per rank against the CPU oracle."""
    Lr = (Lb + 127) // 128 * 128
    src = torch.empty(G * k * Lb, dtype=torch.uint8, device=dev)
    rep = torch.zeros(G * r * Lr, dtype=torch.uint8, device=dev)
    L.check(lib.qf_fill_splitmix_dev(ctx.handle, src.data_ptr(), src.numel(), SEED,
                                     payload_word_offset(rank, G, k, Lb)), "fill")
    enc_args = dict(src_row_stride=Lb, src_gen_stride=k * Lb, rep_row_stride=Lr, rep_gen_stride=r * Lr, G=G,
                    zero_tail=True, ctx=ctx)
    fec.encode_batch(src, rep, k, r, Lb, **enc_args)
    erased = erasure_plan(G, k, e, SEED + 0xC4 + rank)
    aidx = arrival_index(erased, k, r)
    n_slots = aidx.shape[1]
    rows = torch.empty(G * n_slots * Lb, dtype=torch.uint8, device=dev)
    srcv, repv, rowsv = src.view(G, k, Lb), rep.view(G, r, Lr)[:, :, :Lb], rows.view(G, n_slots, Lb)
    aidx_t = torch.from_numpy(aidx.astype(np.int64)).to(dev)
    CH = 4096
    for g0 in range(0, G, CH):
        g1 = min(G, g0 + CH)
        both = torch.cat([srcv[g0:g1], repv[g0:g1]], dim=1)
        gi = torch.arange(g1 - g0, device=dev)[:, None].expand(-1, n_slots)
        rowsv[g0:g1] = both[gi, aidx_t[g0:g1]]
        del both
    row_index = torch.from_numpy(aidx.view(np.int16)).to(dev)
    emax = min(k, r)
    rec = torch.empty(G * emax * Lb, dtype=torch.uint8, device=dev)
    rec_index = torch.empty(G * emax, dtype=torch.int16, device=dev)
    n_rec = torch.empty(G, dtype=torch.int32, device=dev)
    status = torch.empty(G, dtype=torch.int32, device=dev)
    dec_args = dict(max_rows=n_slots, row_stride=Lb, rows_gen_stride=n_slots * Lb, rec_row_stride=Lb,
                    rec_gen_stride=emax * Lb, G=G, ctx=ctx)

    # split: the headline's stream plan (the decode's acceptance pass on a
    # second stream beside the encode, its payload pass after the encode)
    ctx_dec, s_dec = ctx, stream
    if split:
        s_dec = torch.cuda.Stream(dev)
        ctx_dec = fec.Context(dev.index if dev.index is not None else 0, s_dec.cuda_stream)
        dec_args["ctx"] = ctx_dec

    def step(ev):
        ev[0].record(stream)
        if split:
            s_dec.wait_event(ev[0])
        fec.encode_batch(src, rep, k, r, Lb, **enc_args)
        ev[1].record(stream)
        if split:
            ctx_dec.set_payload_wait(ev[1])
        fec.decode_batch(rows, row_index, rec, rec_index, n_rec, status, k, r, Lb, **dec_args)
        if split:
            e_d = torch.cuda.Event()
            e_d.record(s_dec)
            stream.wait_event(e_d)
        ev[2].record(stream)

    for _ in range(max(1, warmup)):
        step([torch.cuda.Event(enable_timing=True) for _ in range(3)])
    torch.cuda.synchronize()
    if _pg(dist, world):
        dist.barrier()
    torch.cuda.synchronize()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    ctx.profile(True)
    if split:
        ctx_dec.profile(True)
    t0 = time.perf_counter()
    for s_ in range(steps):
        step(evs[s_])
    torch.cuda.synchronize()
    if _pg(dist, world):
        dist.barrier()
    torch.cuda.synchronize()
    step_ms = (time.perf_counter() - t0) * 1e3 / steps
    kt = ctx.kernel_times()
    ctx.profile(False)
    if split:
        kt.update(ctx_dec.kernel_times())
        ctx_dec.profile(False)
    enc_ms = float(np.mean([a.elapsed_time(b) for a, b, _ in evs]))
    dec_ms = float(np.mean([b.elapsed_time(c) for _, b, c in evs]))
    er_t = torch.from_numpy(erased).to(dev)
    ok = bool((status == 0).all().item()) and bool((n_rec == e).all().item())
    ok &= bool((rec_index.view(G, emax)[:, :e].long() == er_t).all().item())
    for g0 in range(0, G, 16384):     # recovered bytes, in slices (no G x e x L temporary)
        g1 = min(G, g0 + 16384)
        gi = torch.arange(g0, g1, device=dev)[:, None].expand(-1, e)
        ok &= bool((rec.view(G, emax, Lb)[g0:g1, :e] == srcv[gi, er_t[g0:g1]]).all().item())
    ok &= bool((rep.view(G, r, Lr)[:, :, Lb:] == 0).all().item())
    sample_ok = True
    if rank_sample > 0:
        sample_ok = rank_oracle_sample(torch, src, rep, rows, aidx, rec, k, r, Lb, Lr, e, G, rank_sample,
                                       SEED + 0xC4 + rank)
    cdev = dev if backend == "nccl" else "cpu"
    step_max, enc_max, dec_max, bad = reduce_max(torch, dist, [step_ms, enc_ms, dec_ms,
                                                               0.0 if ok and sample_ok else 1.0], world, cdev)
    src_total = world * G * k * Lb
    del src, rep, rows, rec, rec_index, n_rec, status, row_index, aidx_t
    torch.cuda.empty_cache()
    if split:
        ctx_dec.close()
    return {"workload": f"C4: {G:,} generations = {G * k:,} packets of {Lb} B per rank, encode (r={r}, zero-tail "
                        f"repair rows) then decode with {e} erased sources per generation; independent generations "
                        f"sharded over {world} rank(s), no data-path collective",
            "generations_per_rank": G, "packets_per_rank": G * k, "ranks": world, "steps": steps,
            "value": round(src_total / (step_max / 1e3) / 2**30, 3), "unit": "GiB/s",
            "ms_per_step": round(step_max, 4), "encode_ms": round(enc_max, 4), "decode_ms": round(dec_max, 4),
            "encode_gibps": round(src_total / (enc_max / 1e3) / 2**30, 3),
            "decode_gibps": round(src_total / (dec_max / 1e3) / 2**30, 3),
            "kernel_ms_per_launch": {n: round(ms / max(1, c), 4) for n, (c, ms) in kt.items()},
            "schedule": "split" if split else "serial",
            "oracle_sample_generations_per_rank": rank_sample, "verified": bad == 0}


def c5_leg(fec, ctx, mixed_bytes: float, shape_bytes: float, reps: int = 3) -> dict:
    """BASELINE configs[4] (adaptive.rs:124-153 / 519-562):
    ASW-RLNC-X windows k = 32..196 at 9,000-B jumbo rows, r = ceil(k ratio) - k.
    One heterogeneous batch of all seven shapes (qf_encode_batch_desc /
    qf_decode_batch_desc, >= 4 GB of source, every recovered row verified on
    the device), then per shape block encode, block decode at 20 % loss and
    sliding encode (one window per source packet).  Bytes: block (k + r) L,
    decode (k + e) L, sliding (1 + r) L per window with its VALU fraction
    (compute-bound by construction).  Outside the headline's timed steps."""
    import sys

    sys.path.insert(0, str(REPO / "tools"))
    import bench_c5

    t0 = time.perf_counter()
    res = bench_c5.c5_bench(fec, ctx, mixed_bytes, shape_bytes, reps)
    res["seconds"] = round(time.perf_counter() - t0, 1)
    return res


def gather_flags(torch, dist, flag: int, world: int, device) -> list:
    """Every rank's small integer flag (RCCL all_gather)."""
    t = torch.tensor([flag], dtype=torch.int64, device=device)
    if not _pg(dist, world):
        return [flag]
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [int(x.item()) for x in out]


def rank_oracle_sample(torch, src, rep, rows, aidx, rec, k, r, Lb, Lr, e, G, n, seed) -> bool:
    """C4 verification: n seeded generations of this rank,
    encode and decode, checked against the CPU oracle (outside the timed
    region)."""
    import sys

    sys.path.insert(0, str(REPO))
    from tests import oracle_py as oracle  # test infrastructure: checker only

    gens = np.random.default_rng(seed).choice(G, size=min(n, G), replace=False)
    n_slots = aidx.shape[1]
    emax = min(k, r)
    srcv, repv = src.view(G, k, Lb), rep.view(G, r, Lr)
    rowsv, recv = rows.view(G, n_slots, Lb), rec.view(G, emax, Lb)
    ok = True
    for g in gens.tolist():
        s_h = srcv[g].cpu().numpy()
        ok &= bool((oracle.encode(s_h, r) == repv[g, :, :Lb].cpu().numpy()).all())
        st, sol, mask = oracle.decode(k, aidx[g], rowsv[g].cpu().numpy())
        er = np.nonzero(mask == 0)[0]
        ok &= st == 0 and len(er) == e and bool((sol[er] == recv[g, :e].cpu().numpy()).all())
    return bool(ok)


def sliding_halo_leg(torch, dist, ctx, lib, L, rank, world, dev, backend, packets=65536, k=64, r=10, Lb=1200,
                     reps=5):
    """The sliding-window stream sharded over the ranks: each
    rank receives the k - 1 packet halo of its predecessor over the process
    group (RCCL send/recv over xGMI under nccl) and encodes one window per
    own packet.  Timed (halo + encode, max over ranks) and verified: every
    rank's first window must equal the encode of the global stream's packets."""
    from quicfuscate_amd import fec
    from quicfuscate_amd import stream_shard as ss

    stride = (Lb + 15) // 16 * 16
    P = packets * world
    lo, hi = ss.packet_range(P, rank, world)
    rows_s = torch.empty((hi - lo, stride), dtype=torch.uint8, device=dev)
    L.check(lib.qf_fill_splitmix_dev(ctx.handle, rows_s.data_ptr(), rows_s.numel(), SEED, lo * stride // 8), "fill")
    first, nwin = ss.local_windows(lo, hi, k)
    rep_s = torch.empty(max(1, nwin) * r * stride, dtype=torch.uint8, device=dev)

    def step():
        ext = ss.halo_exchange(torch, dist, rows_s, k, rank, world)
        ss.encode_sliding_local(ext, lo, hi, k, r, Lb, rep_s, rep_row_stride=stride, ctx=ctx)
        return ext

    step()
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        ext = step()
    torch.cuda.synchronize()
    dist.barrier()
    ms = (time.perf_counter() - t0) * 1e3 / reps
    # the first window of this rank (global packets first-k+1 .. first) rebuilt from the global stream
    want_rows = torch.empty((k, stride), dtype=torch.uint8, device=dev)
    L.check(lib.qf_fill_splitmix_dev(ctx.handle, want_rows.data_ptr(), want_rows.numel(), SEED,
                                     (first - k + 1) * stride // 8), "fill")
    want = torch.empty(r * stride, dtype=torch.uint8, device=dev)
    fec.encode_batch(want_rows.view(-1), want, k, r, Lb, src_row_stride=stride, src_gen_stride=k * stride,
                     rep_row_stride=stride, rep_gen_stride=r * stride, G=1, ctx=ctx)
    ctx.sync()
    ok = bool(torch.equal(want.view(r, stride)[:, :Lb], rep_s.view(-1, r, stride)[0, :, :Lb]))
    cdev = dev if backend == "nccl" else "cpu"
    t = torch.tensor([ms, 0.0 if ok else 1.0], dtype=torch.float64, device=cdev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ms_max, bad = t.tolist()
    return {"packets_per_rank": packets, "k": k, "r": r, "L": Lb, "halo_packets": k - 1,
            "backend": dist.get_backend(), "ms_per_step_max": round(ms_max, 4),
            "windows_per_s": round(P / (ms_max / 1e3), 1), "first_window_matches": bad == 0}


def c3_bernoulli_leg(torch, fec, ctx, srcv, repv, k, r, Lb, G, dev, p_loss=0.2, reps=3) -> dict:
    """SURVEY 8(d) C3 secondary variant: every one of the k + r rows of a
    generation is lost i.i.d. with p = 0.2; arrivals are the surviving sources
    in index order, then the surviving repairs.  A generation decodes iff at
    least k rows arrive (decoder.rs:679); the success rate is compared with
    the row counts and with P(Binom(k + r, p) <= r), and every recovered byte
    with the source it replaces."""
    import math

    n = k + r
    rng = np.random.default_rng(SEED ^ 0xB3)
    keep = rng.random((G, n)) >= p_loss
    n_rows = keep.sum(axis=1).astype(np.int32)
    order = np.argsort(~keep, axis=1, kind="stable")          # kept rows first, in index order
    aidx = np.where(np.arange(n)[None, :] < n_rows[:, None], order, 0).astype(np.uint16)
    rows = torch.empty(G * n * Lb, dtype=torch.uint8, device=dev)
    rowsv = rows.view(G, n, Lb)
    aidx_t = torch.from_numpy(aidx.astype(np.int64)).to(dev)
    CH = 4096
    for g0 in range(0, G, CH):
        g1 = min(G, g0 + CH)
        both = torch.cat([srcv[g0:g1], repv[g0:g1]], dim=1)
        gi = torch.arange(g1 - g0, device=dev)[:, None].expand(-1, n)
        rowsv[g0:g1] = both[gi, aidx_t[g0:g1]]
        del both
    row_index = torch.from_numpy(aidx.view(np.int16)).to(dev)
    n_rows_t = torch.from_numpy(n_rows).to(dev)
    emax = min(k, r)
    rec = torch.empty(G * emax * Lb, dtype=torch.uint8, device=dev)
    rec_index = torch.empty(G * emax, dtype=torch.int16, device=dev)
    n_rec = torch.empty(G, dtype=torch.int32, device=dev)
    status = torch.empty(G, dtype=torch.int32, device=dev)
    args = dict(max_rows=n, row_stride=Lb, rows_gen_stride=n * Lb, rec_row_stride=Lb, rec_gen_stride=emax * Lb, G=G,
                n_rows=n_rows_t, ctx=ctx)

    def dec():
        fec.decode_batch(rows, row_index, rec, rec_index, n_rec, status, k, r, Lb, **args)

    dec()
    torch.cuda.synchronize()
    ctx.profile(True)
    for _ in range(reps):
        dec()
    torch.cuda.synchronize()
    kt = ctx.kernel_times()
    ctx.profile(False)
    dec_ms = sum(ms for _, ms in kt.values()) / reps
    st = status.cpu().numpy()
    ok = st == 0
    expect = n_rows >= k
    # recovered rows: the sources that did not arrive (all arrivals that are
    # sources come first, so every received source is accepted)
    nr = n_rec.cpu().numpy()
    verified = bool((ok == expect).all() and (nr[ok] == (k - keep[ok, :k].sum(axis=1))).all()
                    and ((st[~ok] == -3).all()))
    if verified and ok.any():
        ri = rec_index.view(G, emax).long()
        gsel = torch.from_numpy(np.nonzero(ok)[0]).to(dev)
        m = torch.from_numpy(np.arange(emax)[None, :] < nr[ok][:, None]).to(dev)
        got = rec.view(G, emax, Lb)[gsel]
        want = srcv[gsel[:, None].expand(-1, emax), ri[gsel].clamp(0, k - 1)]
        verified = bool(((got == want) | ~m[..., None]).all().item())
    p_ok = sum(math.comb(n, j) * p_loss ** j * (1 - p_loss) ** (n - j) for j in range(0, r + 1))
    src_bytes = float(ok.sum()) * k * Lb
    return {"generations": G, "loss": p_loss, "rows_per_generation": n,
            "success_rate": round(float(ok.mean()), 4), "expected_success_rate": round(p_ok, 4),
            "success_iff_k_rows_arrived": bool((ok == expect).all()), "verified": verified,
            "decode_ms": round(dec_ms, 4), "kernels": {n_: round(ms / reps, 4) for n_, (c, ms) in kt.items()},
            "decode_gibps_source_of_decoded_generations": round(src_bytes / (dec_ms / 1e3) / 2**30, 1)}


def host_path_rate(torch, lib, L, ctx, k, r, Lb, G):
    """Pinned host -> H2D -> encode -> D2H rate (reported in DESIGN.md; never `value`)."""
    import ctypes

    src_h = torch.empty(G * k * Lb, dtype=torch.uint8, pin_memory=True)
    rep_h = torch.empty(G * r * Lb, dtype=torch.uint8, pin_memory=True)
    src_h.copy_(torch.randint(0, 256, (G * k * Lb,), dtype=torch.uint8))
    sh = L.EncodeShape(k, r, Lb, 0, Lb, k * Lb, Lb, r * Lb)
    L.check(lib.qf_encode_batch_host(ctx.handle, ctypes.byref(sh), G, src_h.data_ptr(), rep_h.data_ptr(), None))
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        L.check(lib.qf_encode_batch_host(ctx.handle, ctypes.byref(sh), G, src_h.data_ptr(), rep_h.data_ptr(), None))
    dt = (time.perf_counter() - t0) / reps
    # the same generations through the device-resident encode (qf_encode_batch)
    src_d = src_h.cuda()
    rep_d = torch.empty(G * r * Lb, dtype=torch.uint8, device="cuda")
    L.check(lib.qf_encode_batch(ctx.handle, ctypes.byref(sh), G, src_d.data_ptr(), rep_d.data_ptr(), None))
    ctx.sync()
    same = bool(torch.equal(rep_d.cpu(), rep_h))
    del src_d, rep_d
    return {"generations": G, "encode_src_gibps_incl_pcie": round(G * k * Lb / dt / (1 << 30), 3),
            "bytes_moved_gb": round(G * (k + r) * Lb / 1e9, 3), "seconds": round(dt, 4),
            "matches_device_encode": same}


def host_decode_rate(torch, lib, L, ctx, rows, row_index, rec, e, n_slots, k, r, Lb, G):
    """Pinned host rows -> H2D -> decode -> D2H recovered rows
    (qf_decode_batch_host); results compared with the device decode of the
    same generations.  Reported in DESIGN.md; never `value`."""
    import ctypes

    emax = min(k, r)
    rows_h = torch.empty(G * n_slots * Lb, dtype=torch.uint8, pin_memory=True)
    rows_h.copy_(rows[: G * n_slots * Lb])
    idx_h = torch.empty(G * n_slots, dtype=torch.int16, pin_memory=True)
    idx_h.copy_(row_index[:G].reshape(-1))
    rec_h = torch.empty(G * emax * Lb, dtype=torch.uint8, pin_memory=True)
    ridx_h = torch.empty(G * emax, dtype=torch.int16, pin_memory=True)
    nrec_h = torch.empty(G, dtype=torch.int32, pin_memory=True)
    st_h = torch.empty(G, dtype=torch.int32, pin_memory=True)
    sh = L.DecodeShape(k, r, Lb, n_slots, Lb, n_slots * Lb, Lb, emax * Lb)

    def run():
        L.check(lib.qf_decode_batch_host(ctx.handle, ctypes.byref(sh), G, rows_h.data_ptr(), idx_h.data_ptr(), None,
                                         None, rec_h.data_ptr(), ridx_h.data_ptr(), nrec_h.data_ptr(),
                                         st_h.data_ptr()), "decode_batch_host")

    run()
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        run()
    dt = (time.perf_counter() - t0) / reps
    got = rec_h.view(G, emax, Lb)[:, :e]
    want = rec[: G * emax * Lb].view(G, emax, Lb)[:, :e].cpu()
    ok = bool((st_h == 0).all()) and bool((got == want).all())
    return {"generations": G, "decode_src_gibps_incl_pcie": round(G * k * Lb / dt / (1 << 30), 3),
            "bytes_moved_gb": round(G * (n_slots + e) * Lb / 1e9, 3), "seconds": round(dt, 4),
            "matches_device_decode": ok}


def cpu_variants(src, rep, k, r, Lb, S):
    """SURVEY 8(d) CPU comparison encoders (oracle/cpu_variants.c), encode
    only, at 1 thread, at the box's per-GPU CPU share (16) and at every CPU
    this process may run on:
      table           the reference's loop (decoder.rs:228-259) with table gf_mul;
      clmul_dispatch  the reference AS WRITTEN: per byte gf_mul ->
                      dispatch_bitslice (FeatureDetector + HashMap lookups,
                      optimize.rs:385-408) -> PCLMULQDQ + fold (gf_tables.rs:76-141);
      clmul           the same product without the dispatch (a lower bound on
                      the reference's cost); both clmul outputs are wrong
                      (SURVEY F3), timing only;
      avx2            split-nibble pshufb;  gfni  AVX-512 GF2P8AFFINEQB (0x11D matrices).
    Outputs of table/avx2/gfni are checked against the GPU repairs of the same
    sample.  Reported beside cpu_baseline, not instead."""
    import sys

    sys.path.insert(0, str(REPO))
    from tests import oracle_py as oracle  # test infrastructure

    src_h = src[: S * k * Lb].cpu().numpy().reshape(S, k, Lb)
    rep_h = rep[: S * r * Lb].cpu().numpy().reshape(S, r, Lb)
    try:
        n_all = len(os.sched_getaffinity(0))
    except AttributeError:
        n_all = os.cpu_count() or 1
    thread_counts = sorted({1, min(16, n_all), n_all})
    res = {"threads_available": n_all, "cpu_count": os.cpu_count(), "thread_counts": thread_counts,
           "note": "the GPU box allots 16 CPUs per GPU; the all-CPU rows time-share whatever the box grants",
           "unit": "GiB/s (source payload, encode)", "cpu_model": _cpu_model()}
    # generations per timed call: slow kinds use fewer at 1 thread
    per_gen_s = {"table": 1.6e-3, "clmul": 3.3e-3, "clmul_dispatch": 0.06}
    for kind in ("table", "clmul_dispatch", "clmul", "avx2", "gfni"):
        if not oracle.has_cpu_kind(kind):
            res[kind] = f"no {kind} on this host"
            continue
        for nt in thread_counts:
            # about 1 s of work per call at most, and enough generations per thread
            n = S
            if kind in per_gen_s:
                n = int(max(nt, min(S, 1.0 * nt / per_gen_s[kind])))
            reps, t0 = 0, time.perf_counter()
            while True:   # repeat fast variants until >= 0.25 s so the rate is not a timer artefact
                got = oracle.cpu_encode(kind, src_h[:n], r, nt)
                reps += 1
                dt = time.perf_counter() - t0
                if dt >= 0.25:
                    break
            ent = {"gibps": round(reps * n * k * Lb / dt / (1 << 30), 4), "generations": n, "reps": reps,
                   "seconds": round(dt, 3), "matches_gpu": bool((got == rep_h[:n]).all())}
            if kind == "clmul":
                ent["note"] = "reference product as written WITHOUT its per-byte dispatch: lower bound, timing only"
            if kind == "clmul_dispatch":
                ent["note"] = "reference as written incl. per-byte FeatureDetector/HashMap dispatch, timing only (F3)"
            res[f"{kind}_{nt}t"] = ent
    return res


ISA_FLAGS = ("sse2", "ssse3", "avx", "avx2", "avx512f", "avx512bw", "avx512vbmi", "avx512vl", "gfni", "pclmulqdq",
             "vpclmulqdq", "vaes")


def cpu_host() -> dict:
    """the host the CPU rows ran on -- model, the
    ISA flags the variants use, CPUs visible / usable, thread pinning."""
    flags = set()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("flags"):
                    flags = set(line.split(":", 1)[1].split())
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    return {"cpu_model": _cpu_model(), "nproc": os.cpu_count(), "usable_cpus": usable,
            "cgroup_cpu_quota": cgroup_cpu_quota(),
            "isa_flags": [f for f in ISA_FLAGS if f in flags],
            "pinning": "worker w pinned to the w-th CPU of this process's affinity mask (pthread_attr_setaffinity_np) "
                       "for the cpu_c1 rows; cpu_variants unpinned; cpu_baseline single-threaded"}


def cpu_c1(torch, fec, ctx, Lb, seconds=1.5):
    """BASELINE C1: the reference's CPU encode at its own shape,
    k = 16 sources of L bytes, r in {16, 1} (adaptive.rs:139 Light = (16, 17);
    tests/fec.rs:20-50), 0 % loss (the decoder passes the systematic rows
    through), on 1 thread and on the 16 CPUs the box grants per GPU, threads
    pinned.  Kinds: "table" = the reference's loop (decoder.rs:228-259) with
    gf_mul_table semantics (the port); "clmul_dispatch" = the reference as
    written (per-byte dispatch + CLMUL fold, timing only); "gfni" =
    an optimized host encoder.  Every output that should equal the GPU's is
    compared with the GPU encode of the same generations."""
    import sys

    sys.path.insert(0, str(REPO))
    from tests import oracle_py as oracle  # test infrastructure: CPU baseline only

    k = 16
    rng = np.random.default_rng(SEED ^ 0xC1)
    try:
        n_all = len(os.sched_getaffinity(0))
    except AttributeError:
        n_all = os.cpu_count() or 1
    threads = sorted({1, min(16, n_all)})
    res = {"shape": f"k={k}, L={Lb}, r in (16, 1), 0 % loss (encode; decode passes systematic rows through)",
           "unit": "GiB/s (source payload, encode)", "pinned": True, "thread_counts": threads}
    oracle.set_pinning(True)
    per_gen_s = {"table": 1.2e-3, "clmul_dispatch": 20e-3, "gfni": 1e-5}
    for r in (16, 1):
        Gs = 4096
        src = rng.integers(0, 256, (Gs, k, Lb), dtype=np.uint8)
        # the same generations on the GPU (checker for the CPU outputs)
        d_src = torch.from_numpy(src.reshape(-1)).cuda()
        d_rep = torch.empty(Gs * r * Lb, dtype=torch.uint8, device="cuda")
        fec.encode_batch(d_src, d_rep, k, r, Lb, src_row_stride=Lb, src_gen_stride=k * Lb, rep_row_stride=Lb,
                         rep_gen_stride=r * Lb, G=Gs, ctx=ctx)
        ctx.sync()
        gpu = d_rep.cpu().numpy().reshape(Gs, r, Lb)
        del d_src, d_rep
        for kind in ("table", "clmul_dispatch", "gfni"):
            if not oracle.has_cpu_kind(kind):
                res[f"{kind}_r{r}"] = f"no {kind} on this host"
                continue
            for nt in threads:
                # about `seconds` of work per row, at least one generation per thread
                n = int(max(nt, min(Gs, seconds * nt / (per_gen_s[kind] * r / 16))))
                t0 = time.perf_counter()
                got = oracle.cpu_encode(kind, src[:n], r, nt)
                dt = time.perf_counter() - t0
                ent = {"gibps": round(n * k * Lb / dt / (1 << 30), 5), "generations": n, "seconds": round(dt, 3)}
                if kind == "clmul_dispatch":
                    ent["note"] = "reference as written (defective fold, SURVEY F3): timing only"
                else:
                    ent["matches_gpu"] = bool((got == gpu[:n]).all())
                res[f"{kind}_r{r}_{nt}t"] = ent
    oracle.set_pinning(False)
    return res


def cpu_gf_mul_loop(target_s=0.3):
    """The reference's only published numbers (BASELINE.md section 1:
    docs/gf_bitslice_bench.md 850-4,800 MB/s) come from this 1,024-pair
    gf_mul micro-loop (benches/gf_bitslice_bench.rs:17-102); restated in
    oracle/cpu_variants.c cpu_gf_mul_loop and timed here, one thread, so they
    have a same-host counterpart.  MB/s = 1,024 products (bytes) per pass."""
    import sys

    sys.path.insert(0, str(REPO))
    from tests import oracle_py as oracle

    res = {"unit": "MB/s (10^6 products/s, one thread)", "published_mb_s": {
        "SSE2 table": 850, "AVX2 bit-sliced": 3000, "AVX-512 bit-sliced": 4800, "scalar fallback": 750}}
    for kind in ("table", "dispatch", "sse2", "avx2", "avx512"):
        iters, dt = 64, 0.0
        while True:
            t0 = time.perf_counter()
            acc = oracle.gf_mul_loop(kind, iters)
            dt = time.perf_counter() - t0
            if acc < 0 or dt >= target_s or iters >= 1 << 26:
                break
            iters *= 4
        res[kind] = "not available on this host" if acc < 0 else {
            "mb_s": round(1024 * iters / dt / 1e6, 1), "passes": iters, "seconds": round(dt, 3), "acc": acc}
    res["note"] = ("table = gf_mul_table; dispatch = gf_mul through dispatch_bitslice (the reference's gf_mul); "
                   "sse2 / avx2 / avx512 = the CLMUL-fold members called directly, gf_tables.rs:129-141 / 102-118 / "
                   "76-94 (defective fold, SURVEY F3)")
    return res


def copy_bandwidth(torch, nbytes=4 << 30, reps=5):
    """a device-to-device copy of the same order of bytes as one
    encode launch, for context beside the roofline (read + write bytes / time;
    outside the timed steps, never `value`)."""
    a = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    b = torch.empty_like(a)
    a.fill_(1)
    b.copy_(a)
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0.record()
    for _ in range(reps):
        b.copy_(a)
    t1.record()
    torch.cuda.synchronize()
    ms = t0.elapsed_time(t1) / reps
    del a, b
    torch.cuda.empty_cache()
    return {"bytes_per_copy": nbytes, "ms": round(ms, 4), "gbps_read_plus_write": round(2 * nbytes / (ms / 1e3) / 1e9, 1),
            "note": "torch device-to-device copy (hipMemcpy-class), context only"}


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(src, rep, rows, aidx, rec, n_rec, rec_index, k, r, Lb, e, S):
    """The CPU oracle (port of the reference's loops) on the first S benchmark
    generations, and its outputs checked against the GPU's on that sample:
      single core  the scalar port: encode decoder.rs:172-275 (table gf_mul),
                   Gauss-Jordan decode decoder.rs:720-783 (F4 fixed), one thread;
      all cores    the same encode and decode (oracle/cpu_variants.c) with the
                   generations split over every CPU this process may use, one
                   generation per pinned thread at a time (the reference fans a
                   decode's row operations out on rayon, decoder.rs:410-433,
                   479-489: one generation per core is at least as parallel);
                   also at the 16 CPUs the box allots per GPU;
      as written   encode + decode with every product through the reference's
                   gf_mul -> dispatch_bitslice -> CLMUL fold (optimize.rs:385-408,
                   gf_tables.rs:76-141) on all cores: its per-byte cost; its
                   output is the defective fold, timing only.
    `value` / `cores` are the all-core table figure (encode + decode of the
    sample's source bytes); the single-core figure stays beside it."""
    import sys

    sys.path.insert(0, str(REPO))
    from tests import oracle_py as oracle  # test infrastructure: baseline + sample check only

    src_h = src[: S * k * Lb].cpu().numpy().reshape(S, k, Lb)
    rep_h = rep[: S * r * Lb].cpu().numpy().reshape(S, r, Lb)
    n_slots = aidx.shape[1]
    rows_h = rows[: S * n_slots * Lb].cpu().numpy().reshape(S, n_slots, Lb)
    ri_h = np.ascontiguousarray(np.asarray(aidx[:S]), dtype=np.uint16)
    emax = min(k, r)
    rec_h = rec[: S * emax * Lb].cpu().numpy().reshape(S, emax, Lb)
    erased = []   # per generation: the source rows the decode recovers (the oracle's received mask)
    parity = True
    t0 = time.perf_counter()
    for g in range(S):
        want = oracle.encode(src_h[g], r)
        parity &= bool((want == rep_h[g]).all())
    t_enc = time.perf_counter() - t0
    t0 = time.perf_counter()
    for g in range(S):
        st, sol, mask = oracle.decode(k, aidx[g], rows_h[g])
        er = np.nonzero(mask == 0)[0]
        erased.append(er)
        parity &= st == 0 and bool((sol[er] == rec_h[g, : len(er)]).all())
    t_dec = time.perf_counter() - t0
    src_bytes = S * k * Lb
    try:
        n_all = len(os.sched_getaffinity(0))
    except AttributeError:
        n_all = os.cpu_count() or 1
    # the CPUs this process may actually keep busy: the affinity mask, capped by
    # the cgroup's CPU quota (the GPU box's mask shows the whole host, 256 CPUs,
    # under a quota of 16 per GPU)
    quota = cgroup_cpu_quota()
    usable = min(n_all, quota) if quota else n_all

    def timed(fn, min_s=1.0):
        reps, t0 = 0, time.perf_counter()
        while True:
            out = fn()
            reps += 1
            dt = time.perf_counter() - t0
            if dt >= min_s:
                return out, dt / reps

    oracle.set_pinning(True)
    legs = {}
    for nt in sorted({min(16, n_all), usable, n_all}):
        got_rep, te = timed(lambda: oracle.cpu_encode("table", src_h, r, nt))
        got_dec, td = timed(lambda: oracle.cpu_decode("table", k, ri_h, rows_h, nt))
        ok = bool((got_rep == rep_h).all())
        for g in range(S):
            ok &= bool((got_dec[g][erased[g]] == rec_h[g, : len(erased[g])]).all())
        legs[nt] = {"value": round(src_bytes / (te + td) / (1 << 30), 4), "cores": nt,
                    "encode_gibps": round(src_bytes / te / (1 << 30), 4),
                    "decode_gibps": round(src_bytes / td / (1 << 30), 4), "sample_parity_vs_gpu": ok}
    as_written = None
    if oracle.has_cpu_kind("clmul_dispatch"):
        n = min(S, max(n_all, 4 * n_all))   # about 1 s per leg on a 64-core host
        _, te = timed(lambda: oracle.cpu_encode("clmul_dispatch", src_h[:n], r, n_all), 0.5)
        _, td = timed(lambda: oracle.cpu_decode("clmul_dispatch", k, ri_h[:n], rows_h[:n], n_all), 0.5)
        b = n * k * Lb
        as_written = {"value": round(b / (te + td) / (1 << 30), 4), "cores": n_all, "generations": n,
                      "encode_gibps": round(b / te / (1 << 30), 4), "decode_gibps": round(b / td / (1 << 30), 4),
                      "note": "per-byte dispatched CLMUL-fold products (the reference as written): timing only, "
                              "SURVEY F3"}
    oracle.set_pinning(False)
    allc = legs[usable]
    single = {"value": round(src_bytes / (t_enc + t_dec) / (1 << 30), 5), "cores": 1,
              "encode_gibps": round(src_bytes / t_enc / (1 << 30), 5),
              "decode_gibps": round(src_bytes / t_dec / (1 << 30), 5), "seconds": round(t_enc + t_dec, 2),
              "sample_parity_vs_gpu": bool(parity)}
    return {
        "value": allc["value"],
        "unit": "GiB/s",
        "cores": usable,
        "kind": "port",
        "sample": f"first {S} of the benchmark generations: oracle encode (decoder.rs:172-275 loop, table gf_mul) "
                  f"+ oracle Gauss-Jordan decode (decoder.rs:720-783, F4 fixed); all {usable} usable CPUs "
                  f"({n_all} in the affinity mask, cgroup CPU quota {quota or 'none'}), generations split over "
                  f"pinned threads (single-core and whole-mask figures beside)",
        "affinity_cpus": n_all,
        "cgroup_cpu_quota": quota,
        "encode_gibps": allc["encode_gibps"],
        "decode_gibps": allc["decode_gibps"],
        "sample_parity_vs_gpu": bool(parity) and all(v["sample_parity_vs_gpu"] for v in legs.values()),
        "single_core": single,
        "all_cores": allc,
        "affinity_all": legs[n_all],
        "share_16": legs[min(16, n_all)],
        "as_written_all_cores": as_written,
    }


# ---------------------------------------------------------------------------
# The stdout line.  The driver parses ONE JSON line; round 4's full record
# (20.8 KB, c5 / cpu legs verbatim) was not parsed.  The
# line carries the contract keys first, then one compact figure per leg; the
# full record goes to --detail (a file, kept under profiles/ by the builder).
# ---------------------------------------------------------------------------
LINE_MAX = 6000   # bytes; the driver's stdout tail holds ~8 KB


def emit_detail(full: dict, path: str) -> str | None:
    """Write the full per-leg record; returns the path written (or None)."""
    if not path:
        return None
    try:
        p = Path(path)
        if not p.is_absolute():
            p = REPO / p
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(json.dumps(full, indent=1))
        return str(Path(path))
    except OSError:
        return None


def _r(x, nd=1):
    return None if x is None else round(float(x), nd)


def _roof_compact(rl: dict | None) -> dict | None:
    if not rl:
        return None
    out = {k: rl.get(k) for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "launch_ms",
                                  "algorithmic_bytes_per_launch", "limiter")}
    if rl.get("traffic") is not None and rl.get("algorithmic_bytes_per_launch"):
        out["traffic_over_alg"] = round(rl["traffic"] / rl["algorithmic_bytes_per_launch"], 3)
    v = rl.get("valu")
    if v:
        out["valu_frac"] = v.get("frac")
        out["valu_per_wave"] = v.get("valu_per_wave")
    if rl.get("in_step"):
        out["in_step"] = {k: rl["in_step"].get(k) for k in ("launch_ms", "frac")}
    out["timing"] = "HIP events on the launch stream, per launch, inside bench.py"
    if rl.get("timing"):
        out["timing"] = "alone: 5 launches after the timed steps (HIP events); in_step: inside the timed steps"
    out["traffic_src"] = "profiles/traffic.json (rocprofv3 --pmc, same code hash)" if rl.get("traffic") else None
    return out


def _c5_compact(c5: dict | None) -> dict | None:
    """Per shape [block encode, block decode, sliding encode] GiB/s (kernel
    time), the mixed batch's device span beside its kernel sum."""
    if not c5:
        return None
    out = {"L": c5.get("L"), "unit": "GiB/s algorithmic bytes",
           "cols": ["block_enc", "block_dec", "sliding_enc", "block_enc_hbm_frac", "block_dec_hbm_frac",
                    "sliding_valu_frac"]}
    shapes, ok, sources = {}, True, set()
    for key, v in c5.items():
        if not (key.startswith("k") and isinstance(v, dict)):
            continue
        be, bd, sl = v.get("block/encode", {}), v.get("block/decode", {}), v.get("sliding/encode", {})
        sv = sl.get("valu") or {}
        if sv.get("source"):
            sources.add(sv["source"])
        shapes[key] = [be.get("GiBps_alg"), bd.get("GiBps_alg"), sl.get("GiBps_alg"),
                       be.get("hbm_frac_of_8TBps"), bd.get("hbm_frac_of_8TBps"), sv.get("frac")]
        ok &= bd.get("verified", True) is not False and sl.get("verified", True) is not False
    out["shapes"] = shapes
    # where the sliding VALU issue fractions come from: SQ counters of the same
    # kernels (profiles/c5_sq_counters.json, code hash checked) or the static model
    out["sliding_valu_source"] = "/".join(sorted(sources)) or None
    m = c5.get("mixed_desc_batch")
    if m:
        mx = {"G": m.get("G"), "round_trip_ok": m.get("round_trip_ok")}
        for leg in ("encode", "decode"):
            e = m.get(leg, {})
            mx[leg] = {k: e.get(k) for k in ("span_gibps", "kernel_gibps", "span_ms", "kernel_ms", "span_over_kernel",
                                             "host_call_ms") if k in e}
        out["mixed"] = mx
        ok &= m.get("round_trip_ok") is not False
    out["verified"] = ok
    return out


def compact_line(full: dict, detail: str | None = None) -> dict:
    """The stdout JSON line: contract keys first (metric .. config, roofline,
    cpu_baseline), then one compact figure per leg.  Size-checked by
    tests/test_bench_cpu.py against LINE_MAX on a recorded full run."""
    keys = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config")
    line = {k: full.get(k) for k in keys}
    line["roofline"] = _roof_compact(full.get("roofline"))
    cb = full.get("cpu_baseline")
    if cb:
        line["cpu_baseline"] = {k: cb.get(k) for k in ("value", "unit", "cores", "kind", "sample", "encode_gibps",
                                                       "decode_gibps", "sample_parity_vs_gpu", "affinity_cpus",
                                                       "cgroup_cpu_quota")}
        for leg in ("single_core", "share_16", "affinity_all", "as_written_all_cores"):
            if cb.get(leg):
                line["cpu_baseline"][leg] = {k: cb[leg].get(k) for k in ("value", "cores", "encode_gibps",
                                                                         "decode_gibps")}
    line["roofline_encode"] = _roof_compact(full.get("roofline_encode"))
    for k in ("encode_gibps", "decode_gibps", "encode_ms", "decode_ms", "ms_per_step_median_rank0",
              "kernel_ms_per_launch", "verified", "process_group"):
        if k in full:
            line[k] = full[k]
    line["streams"] = "split" if "2nd stream" in (full.get("streams") or "") else full.get("streams")
    rd = full.get("run_descriptor")
    if rd:
        line["descriptor_matches_by_rank"] = rd.get("matches_by_rank")
    if full.get("repair_xor_fold_by_rank") and len(full["repair_xor_fold_by_rank"]) <= 8:
        line["repair_xor_fold_by_rank"] = full["repair_xor_fold_by_rank"]
    c4 = full.get("c4")
    if c4:
        line["c4"] = {k: c4.get(k) for k in ("generations_per_rank", "ranks", "value", "unit", "ms_per_step",
                                             "encode_gibps", "decode_gibps", "schedule", "verified")}
    if "rank_oracle_sample" in full:
        line["rank_oracle_sample"] = full["rank_oracle_sample"]
    if full.get("sliding_halo"):
        sh = full["sliding_halo"]
        line["sliding_halo"] = {k: sh.get(k) for k in ("backend", "ms_per_step_max", "windows_per_s",
                                                       "first_window_matches")}
    if full.get("c5"):
        line["c5"] = _c5_compact(full["c5"])
    b = full.get("c3_bernoulli")
    if b:
        line["c3_bernoulli"] = {k: b.get(k) for k in ("success_rate", "expected_success_rate", "verified",
                                                      "decode_gibps_source_of_decoded_generations")}
    hp = full.get("host_path")
    if hp:
        line["host_path_gibps_incl_pcie"] = {
            "encode": hp.get("encode_src_gibps_incl_pcie"),
            "decode": (hp.get("decode") or {}).get("decode_src_gibps_incl_pcie"),
            "match": bool(hp.get("matches_device_encode")) and bool((hp.get("decode") or {}).get(
                "matches_device_decode", True))}
    if full.get("hbm_copy_context"):
        line["hbm_copy_gbps"] = full["hbm_copy_context"].get("gbps_read_plus_write")
    cv = full.get("cpu_variants")
    if cv:
        line["cpu_variants_gibps"] = {k: (v.get("gibps") if isinstance(v, dict) else None) for k, v in cv.items()
                                      if k.endswith("t") and k.split("_")[-1][:-1].isdigit()}
        # the clmul kinds restate the reference's defective fold: timing only
        line["cpu_variants_match_gpu"] = all(v.get("matches_gpu", True) for k, v in cv.items()
                                             if isinstance(v, dict) and not k.startswith("clmul"))
    c1 = full.get("cpu_c1")
    if c1:
        line["cpu_c1_gibps"] = {k: (v.get("gibps") if isinstance(v, dict) else None) for k, v in c1.items()
                                if k.endswith("t") and k.split("_")[-1][:-1].isdigit()}
    gl = full.get("cpu_gf_mul_loop")
    if gl:
        line["cpu_gf_mul_loop_mb_s"] = {k: (v.get("mb_s") if isinstance(v, dict) else None) for k, v in gl.items()
                                        if k in ("table", "dispatch", "sse2", "avx2", "avx512")}
    ch = full.get("cpu_host")
    if ch:
        line["cpu_host"] = {"model": ch.get("cpu_model"), "usable_cpus": ch.get("usable_cpus")}
    line["detail"] = detail
    s = json.dumps(line)
    if len(s) > LINE_MAX:   # never again an unparsed line: drop optional legs, largest first
        for k in sorted((k for k in line if k not in keys + ("roofline", "cpu_baseline", "roofline_encode", "verified")),
                        key=lambda k: -len(json.dumps(line[k]))):
            line.pop(k)
            if len(json.dumps(line)) <= LINE_MAX:
                break
    return line


if __name__ == "__main__":
    raise SystemExit(main() or 0)
