"""Sliding-window shard encode on the device (quicfuscate_amd.stream_shard,
SURVEY 8(e)): the windows of a rank's packets, halo included, encoded in one
batched call, equal the oracle's encode of each window (adaptive.rs:519-562)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("lo,hi,k,r,L", [(0, 40, 16, 4, 100), (50, 90, 64, 10, 1200), (7, 30, 8, 3, 48)])
def test_encode_sliding_local_matches_oracle(qf, oracle, gpu_ctx, lo, hi, k, r, L):
    import torch

    from quicfuscate_amd import stream_shard as ss

    rng = np.random.default_rng(lo + hi + k)
    stride = (L + 15) // 16 * 16
    stream = rng.integers(0, 256, (hi, stride), dtype=np.uint8)
    # what halo_exchange hands a rank owning [lo, hi): k - 1 halo rows, then its own
    ext = np.zeros((k - 1 + hi - lo, stride), np.uint8)
    for t in range(lo - (k - 1), hi):
        if t >= 0:
            ext[t - lo + k - 1] = stream[t]
    t_ext = torch.from_numpy(ext).cuda()
    rrs = stride
    first, nwin = ss.local_windows(lo, hi, k)
    rep = torch.full((max(1, nwin) * r * rrs,), 0xA5, dtype=torch.uint8, device="cuda")
    n = ss.encode_sliding_local(t_ext, lo, hi, k, r, L, rep, rep_row_stride=rrs)
    qf.default_context().sync()
    assert n == nwin
    got = rep.cpu().numpy()
    for w, t in enumerate(range(first, first + nwin)):
        want = oracle.encode(np.ascontiguousarray(stream[t - k + 1: t + 1, :L]), r)
        for j in range(r):
            off = (w * r + j) * rrs
            assert (got[off: off + L] == want[j]).all(), (t, j)
