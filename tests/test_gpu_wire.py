"""Wire framing on the device (encoder.rs:18-152): frames byte-equal to the
oracle's restatement of Packet::to_raw (oracle/qf_oracle_wire.c), parse
statuses and payloads equal to the oracle's Packet::from_raw, and frames ->
parse -> decode recovers the sources, with lost, reordered and malformed
frames."""
import ctypes

import numpy as np
import pytest

from quicfuscate_amd import _lib as L

pytestmark = pytest.mark.gpu


def _r16(x):
    return (x + 15) // 16 * 16


def _frame_batch(qf, src, rep, k, r, Lb, G, fs):
    """src / rep: rows of round16(Lb) bytes."""
    import torch

    rs = _r16(Lb)
    frames = torch.full((G * (k + r) * fs,), 0xCC, dtype=torch.uint8, device="cuda")
    flen = torch.zeros(G * (k + r), dtype=torch.int32, device="cuda")
    sh = L.EncodeShape(k, r, Lb, 0, rs, k * rs, rs, r * rs)
    L.check(L._lib().qf_frame_batch_dev(qf.default_context().handle, ctypes.byref(sh), G, src.data_ptr(),
                                        rep.data_ptr(), frames.data_ptr(), fs, flen.data_ptr()), "frame")
    qf.default_context().sync()
    return frames.cpu().numpy().reshape(G, k + r, fs), flen.cpu().numpy().reshape(G, k + r)


@pytest.mark.parametrize("k,r,Lb", [(64, 16, 1200), (4, 2, 8), (7, 5, 33), (16, 1, 1)])
def test_frames_equal_to_raw(qf, oracle, gpu_ctx, k, r, Lb):
    import torch

    rng = np.random.default_rng(k + Lb)
    G = 3
    fs = (3 + k + Lb + 15) // 16 * 16
    src_np = rng.integers(0, 256, (G, k, Lb), dtype=np.uint8)
    rep_np = np.stack([oracle.encode(src_np[g], r) for g in range(G)])
    pad = _r16(Lb) - Lb
    src = torch.from_numpy(np.pad(src_np, ((0, 0), (0, 0), (0, pad))).reshape(-1)).cuda()
    rep = torch.from_numpy(np.pad(rep_np, ((0, 0), (0, 0), (0, pad))).reshape(-1)).cuda()
    frames, flen = _frame_batch(qf, src, rep, k, r, Lb, G, fs)
    C = oracle.cauchy(k, r)
    for g in range(G):
        for i in range(k + r):
            if i < k:
                st, want = oracle.packet_to_raw(True, src_np[g, i].tobytes())
            else:
                st, want = oracle.packet_to_raw(False, rep_np[g, i - k].tobytes(), bytes(C[i - k]))
            assert st == 0
            assert flen[g, i] == len(want)
            assert frames[g, i, : len(want)].tobytes() == want, (g, i)
            assert (frames[g, i, len(want):] == 0xCC).all()


def test_frames_parse_decode_round_trip(qf, oracle, gpu_ctx):
    import torch

    k, r, Lb, G = 64, 16, 1200, 6
    fs = (3 + k + Lb + 15) // 16 * 16
    rng = np.random.default_rng(77)
    src_np = rng.integers(0, 256, (G, k, Lb), dtype=np.uint8)
    rep_np = np.stack([oracle.encode(src_np[g], r) for g in range(G)])
    frames, flen = _frame_batch(qf, torch.from_numpy(src_np.reshape(-1)).cuda(),
                                torch.from_numpy(rep_np.reshape(-1)).cuda(), k, r, Lb, G, fs)
    max_rows = k + r + 8
    rx = np.zeros((G, max_rows, fs), np.uint8)
    rx_len = np.zeros((G, max_rows), np.uint32)
    rx_id = np.zeros((G, max_rows), np.uint64)
    n_fr = np.zeros(G, np.uint32)
    expect = []
    for g in range(G):
        keep = [i for i in range(k + r) if rng.random() > 0.15]
        rng.shuffle(keep)
        arr = []   # (frame bytes, len, id, expected status, row index if valid)
        for i in keep:
            arr.append((frames[g, i], flen[g, i], g * 1000 + i if i >= k else 5 * k + i, 0,
                        i if i < k else i))
        bad = frames[g, k].copy()
        arr.insert(int(rng.integers(0, len(arr) + 1)), (bad, 0, 1, L.QF_EINVAL, None))       # empty
        arr.insert(int(rng.integers(0, len(arr) + 1)), (bad, 2, 1, L.QF_ETOOSMALL, None))    # no coeff length
        arr.insert(int(rng.integers(0, len(arr) + 1)), (bad, 40, 1, L.QF_ETOOSMALL, None))   # coeffs truncated
        wrong = bad.copy()
        wrong[5] ^= 1
        arr.insert(int(rng.integers(0, len(arr) + 1)), (wrong, flen[g, k], 1, L.QF_ERANGE, None))  # not Cauchy
        short_k = bad.copy()
        short_k[2] = k - 1
        arr.insert(int(rng.integers(0, len(arr) + 1)), (short_k, flen[g, k], 1, L.QF_ERANGE, None))
        too_long = frames[g, 0].copy()
        arr.insert(int(rng.integers(0, len(arr) + 1)), (too_long, 1 + Lb + 1, 0, L.QF_EINVAL, None))
        n_fr[g] = len(arr)
        for s, (fb, ln, pid, st, ridx) in enumerate(arr):
            rx[g, s] = fb
            rx_len[g, s] = ln
            rx_id[g, s] = pid
        expect.append(arr)
    dev = "cuda"
    t_fr = torch.from_numpy(rx.reshape(-1)).to(dev)
    t_len = torch.from_numpy(rx_len.view(np.int32).reshape(-1)).to(dev)
    t_id = torch.from_numpy(rx_id.view(np.int64).reshape(-1)).to(dev)
    t_n = torch.from_numpy(n_fr.view(np.int32)).to(dev)
    rows = torch.zeros(G * max_rows * Lb, dtype=torch.uint8, device=dev)
    ridx = torch.zeros(G * max_rows, dtype=torch.int16, device=dev)
    nrows = torch.zeros(G, dtype=torch.int32, device=dev)
    fst = torch.full((G * max_rows,), 99, dtype=torch.int32, device=dev)
    L.check(L._lib().qf_parse_frames_dev(qf.default_context().handle, k, r, Lb, G, max_rows, t_fr.data_ptr(), fs,
                                         t_len.data_ptr(), t_id.data_ptr(), t_n.data_ptr(), rows.data_ptr(), Lb,
                                         max_rows * Lb, ridx.data_ptr(), nrows.data_ptr(), fst.data_ptr()), "parse")
    qf.default_context().sync()
    st = fst.cpu().numpy().reshape(G, max_rows)
    ri = ridx.cpu().numpy().view(np.uint16).reshape(G, max_rows)
    nr = nrows.cpu().numpy()
    rw = rows.cpu().numpy().reshape(G, max_rows, Lb)
    C = oracle.cauchy(k, r)
    for g in range(G):
        valid = [e for e in expect[g] if e[3] == 0]
        assert list(st[g, : n_fr[g]]) == [e[3] for e in expect[g]]
        # every status and payload follows the oracle's Packet::from_raw, plus the
        # batch rules (Cauchy row of this (k, r); payload <= L)
        for s_, (fb, ln, pid, want_st, _) in enumerate(expect[g]):
            os_, osys, oco, opay = oracle.packet_from_raw(fb[:ln].tobytes())
            if os_:
                exp = {oracle.FR_EMPTY: L.QF_EINVAL}.get(os_, L.QF_ETOOSMALL)
            elif not osys and (len(oco) != k or not any(bytes(C[j]) == oco for j in range(r))):
                exp = L.QF_ERANGE
            elif len(opay) > Lb:
                exp = L.QF_EINVAL
            else:
                exp = 0
            assert st[g, s_] == exp == want_st, (g, s_)
        assert nr[g] == len(valid)
        for s, (fb, ln, pid, _, i) in enumerate(valid):
            assert ri[g, s] == (pid % k if i < k else i)
            payload = src_np[g, i] if i < k else rep_np[g, i - k]
            assert (rw[g, s] == payload).all()
            assert rw[g, s].tobytes() == oracle.packet_from_raw(fb[:ln].tobytes())[3].ljust(Lb, b"\0")
    # decode straight from the parsed rows
    emax = min(k, r)
    rec = torch.empty(G * emax * Lb, dtype=torch.uint8, device=dev)
    rec_index = torch.empty(G * emax, dtype=torch.int16, device=dev)
    n_rec = torch.empty(G, dtype=torch.int32, device=dev)
    status = torch.empty(G, dtype=torch.int32, device=dev)
    qf.decode_batch(rows, ridx, rec, rec_index, n_rec, status, k, r, Lb, max_rows=max_rows, row_stride=Lb,
                    rows_gen_stride=max_rows * Lb, rec_row_stride=Lb, rec_gen_stride=emax * Lb, G=G, n_rows=nrows)
    qf.default_context().sync()
    stt, nrec = status.cpu().numpy(), n_rec.cpu().numpy()
    recv = rec.cpu().numpy().reshape(G, emax, Lb)
    idx = rec_index.cpu().numpy().view(np.uint16).reshape(G, emax)
    for g in range(G):
        got_src = {e[4] for e in expect[g] if e[3] == 0 and e[4] < k}
        n_rep = sum(1 for e in expect[g] if e[3] == 0 and e[4] >= k)
        if len(got_src) + n_rep < k:
            assert stt[g] == L.QF_ENOTREADY
            continue
        assert stt[g] == 0
        for m in range(nrec[g]):
            assert (recv[g, m] == src_np[g, idx[g, m]]).all()
