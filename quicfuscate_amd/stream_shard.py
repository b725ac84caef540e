"""Sliding-window encode of one packet stream sharded over ranks (SURVEY 8(e),
"sliding-window mode"): rank r holds a contiguous packet range; its first
k - 1 windows reach back into rank r - 1's packets, so each rank receives a
halo of the k - 1 preceding packets by point-to-point send/recv (RCCL over
xGMI on the GPU ranks, gloo in the CPU tests) and then encodes one window per
own packet in a single batched call (adaptive.rs:519-562: after every source
packet the window of the last k packets emits its repairs).  Windows that
end before the stream holds k packets emit nothing, as generate_repair_packet
returns None there (decoder.rs:177-179).
"""
from __future__ import annotations

from . import fec as qf


def packet_range(P: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous packet range [lo, hi) of a rank."""
    return P * rank // world, P * (rank + 1) // world


def halo_exchange(torch, dist, rows, k: int, rank: int, world: int):
    """rows: (n_local, stride) uint8 packets of this rank.  Returns
    (k - 1 + n_local, stride): the k - 1 packets before this rank's first one
    (zeros on rank 0), then its own.  Needs n_local >= k - 1 on every rank
    but the last (the halo comes from the previous rank only)."""
    n, stride = rows.shape
    h = k - 1
    ext = torch.zeros((h + n, stride), dtype=rows.dtype, device=rows.device)
    ext[h:] = rows
    if world == 1 or h == 0:
        return ext
    # gloo moves host tensors only: stage device rows through the host there
    host = dist.get_backend() == "gloo" and rows.device.type != "cpu"
    # every rank learns whether any sender is short BEFORE the first send /
    # recv: a rank raising alone would leave its successor blocked in recv
    ok = torch.tensor([1 if (rank + 1 == world or n >= h) else 0], dtype=torch.int32,
                      device="cpu" if (host or rows.device.type == "cpu") else rows.device)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if int(ok.item()) == 0:
        raise ValueError("sliding shard smaller than the window halo on some rank")
    if rank + 1 < world:
        out = rows[n - h:].contiguous()
        dist.send(out.cpu() if host else out, dst=rank + 1)
    if rank > 0:
        buf = torch.empty((h, stride), dtype=rows.dtype, device="cpu" if host else rows.device)
        dist.recv(buf, src=rank - 1)
        ext[:h] = buf.to(rows.device) if host else buf
    return ext


def local_windows(lo: int, hi: int, k: int) -> tuple[int, int]:
    """(first window end, number of windows) for packets [lo, hi): one window
    per packet t >= k - 1 (the window is packets t - k + 1 .. t)."""
    first = max(lo, k - 1)
    return first, max(0, hi - first)


def encode_sliding_local(ext, lo: int, hi: int, k: int, r: int, L: int, rep, *, rep_row_stride: int,
                         zero_tail: bool = False, ctx=None) -> int:
    """Repairs of every window ending in [lo, hi) into rep (window-major,
    r rows each).  ext is halo_exchange's output (row stride ext.stride(0)).
    Returns the number of windows encoded."""
    first, nwin = local_windows(lo, hi, k)
    if nwin == 0:
        return 0
    stride = ext.stride(0)
    # ext row 0 is global packet lo - (k - 1); window ending at t starts at
    # packet t - k + 1 = ext row t - lo
    start = ext[first - lo:]
    qf.encode_batch(start, rep, k, r, L, src_row_stride=stride, src_gen_stride=stride,
                    rep_row_stride=rep_row_stride, rep_gen_stride=r * rep_row_stride, G=nwin,
                    zero_tail=zero_tail, ctx=ctx)
    return nwin
