"""Host-memory encode pipeline (qf_encode_batch_host): the send side of
core.rs:252-317 starts from UDP datagrams in host memory.  The library
streams ~64 MiB chunks of generations H2D -> encode -> D2H over three HIP
streams with staging reused per pipe slot, so the cases cover several chunks
with a partial last one, pinned and pageable buffers, and the explicit
coefficient path (whose staging is shared by the pipe slots).  Repairs must
equal the oracle (decoder.rs:172-275) on the checked generations and the
device-resident encode on all of them."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CHUNK = 64 << 20   # the library's chunk size (qf_api.hip qf_encode_batch_host)


def _gens_per_chunk(k, stride):
    return max(1, CHUNK // (k * stride))


def _check_sample(oracle, src_np, rep_np, k, r, Lb, gens, coeff=None):
    for g in gens:
        want = oracle.encode(src_np[g, :, :Lb], r, coeff=coeff, L=Lb)
        assert (rep_np[g, :, :Lb] == want).all(), f"generation {g}"


@pytest.mark.parametrize("pinned", [True, False])
def test_encode_host_multi_chunk_cauchy(qf, oracle, gpu_ctx, pinned):
    import torch

    k, r, Lb = 64, 16, 1200
    per = _gens_per_chunk(k, Lb)
    G = 3 * per + per // 3            # 3 full chunks + a partial one (4 pipe uses of 3 slots)
    src_np = oracle.fill_splitmix(G * k * Lb, 0x51464543).reshape(G, k, Lb)
    src_h = torch.from_numpy(src_np.reshape(-1).copy())
    rep_h = torch.full((G * r * Lb,), 0xA5, dtype=torch.uint8)
    if pinned:
        src_h, rep_h = src_h.pin_memory(), rep_h.pin_memory()
    qf.encode_batch_host(src_h, rep_h, k, r, Lb, src_row_stride=Lb, rep_row_stride=Lb, G=G)
    rep_np = rep_h.numpy().reshape(G, r, Lb)
    # the device-resident encode of the same generations, all of them
    src_d = src_h.cuda()
    rep_d = torch.empty(G * r * Lb, dtype=torch.uint8, device="cuda")
    qf.encode_batch(src_d, rep_d, k, r, Lb, src_row_stride=Lb, src_gen_stride=k * Lb, rep_row_stride=Lb,
                    rep_gen_stride=r * Lb, G=G)
    qf.default_context().sync()
    assert torch.equal(rep_d.cpu(), rep_h.cpu())
    # oracle on the chunk boundaries and a seeded sample
    rng = np.random.default_rng(1)
    gens = sorted({0, per - 1, per, 2 * per - 1, 2 * per, 3 * per - 1, 3 * per, G - 1}
                  | set(rng.integers(0, G, 24).tolist()))
    _check_sample(oracle, src_np, rep_np, k, r, Lb, gens)


def test_encode_host_explicit_coefficients(qf, oracle, gpu_ctx):
    """coeff != NULL: the split tables go through the context's shared staging
    on every pipe slot; r > 16 runs two passes per chunk."""
    import torch

    k, r, Lb = 40, 20, 1024
    per = _gens_per_chunk(k, Lb)
    G = 2 * per + 7
    rng = np.random.default_rng(11)
    coeff = rng.integers(0, 256, (r, k), dtype=np.uint8)
    src_np = rng.integers(0, 256, (G, k, Lb), dtype=np.uint8)
    src_h = torch.from_numpy(src_np.reshape(-1).copy()).pin_memory()
    rep_h = torch.zeros(G * r * Lb, dtype=torch.uint8).pin_memory()
    qf.encode_batch_host(src_h, rep_h, k, r, Lb, src_row_stride=Lb, rep_row_stride=Lb, G=G,
                         coeff=coeff.tobytes())
    rep_np = rep_h.numpy().reshape(G, r, Lb)
    gens = sorted({0, per - 1, per, 2 * per - 1, 2 * per, G - 1} | set(rng.integers(0, G, 10).tolist()))
    _check_sample(oracle, src_np, rep_np, k, r, Lb, gens, coeff=coeff)


@pytest.mark.parametrize("k,r,Lb,stride", [(16, 4, 333, 336), (4, 2, 8, 16), (255, 1, 48, 48)])
def test_encode_host_small_shapes_every_generation(qf, oracle, gpu_ctx, k, r, Lb, stride):
    """Row strides above L: only L bytes of each repair row are written."""
    import torch

    G = 37
    rng = np.random.default_rng(k * 7 + Lb)
    src_np = rng.integers(0, 256, (G, k, stride), dtype=np.uint8)
    src_h = torch.from_numpy(src_np.reshape(-1).copy()).pin_memory()
    rep_h = torch.full((G * r * stride,), 0x5A, dtype=torch.uint8).pin_memory()
    qf.encode_batch_host(src_h, rep_h, k, r, Lb, src_row_stride=stride, rep_row_stride=stride, G=G)
    rep_np = rep_h.numpy().reshape(G, r, stride)
    _check_sample(oracle, src_np, rep_np, k, r, Lb, range(G))
    assert (rep_np[:, :, Lb:] == 0x5A).all()


def test_decode_host_multi_chunk_equals_oracle(qf, oracle, gpu_ctx):
    """qf_decode_batch_host over several chunks with a partial last one."""
    import torch

    k, r, Lb, e = 64, 16, 1200, 13
    n_slots = k - e + r
    per = max(1, CHUNK // (n_slots * Lb))
    G = 2 * per + 11
    rng = np.random.default_rng(3)
    src_np = oracle.fill_splitmix(G * k * Lb, 7).reshape(G, k, Lb)
    src_d = torch.from_numpy(src_np.reshape(-1).copy()).cuda()
    rep_d = torch.empty(G * r * Lb, dtype=torch.uint8, device="cuda")
    qf.encode_batch(src_d, rep_d, k, r, Lb, src_row_stride=Lb, src_gen_stride=k * Lb, rep_row_stride=Lb,
                    rep_gen_stride=r * Lb, G=G)
    rep_np = rep_d.cpu().numpy().reshape(G, r, Lb)
    idx = np.zeros((G, n_slots), np.uint16)
    rows = np.zeros((G, n_slots, Lb), np.uint8)
    for g in range(G):
        er = set(rng.choice(k, e, replace=False).tolist())
        arr = [i for i in range(k) if i not in er] + list(range(k, k + r))
        idx[g] = arr
        rows[g] = [src_np[g, a] if a < k else rep_np[g, a - k] for a in arr]
    rows_h = torch.from_numpy(rows.reshape(-1)).pin_memory()
    idx_h = torch.from_numpy(idx.view(np.int16).reshape(-1)).pin_memory()
    emax = min(k, r)
    rec_h = torch.zeros(G * emax * Lb, dtype=torch.uint8).pin_memory()
    ridx_h = torch.zeros(G * emax, dtype=torch.int16).pin_memory()
    nrec_h = torch.zeros(G, dtype=torch.int32).pin_memory()
    st_h = torch.full((G,), 99, dtype=torch.int32).pin_memory()
    qf.decode_batch_host(rows_h, idx_h, rec_h, ridx_h, nrec_h, st_h, k, r, Lb, max_rows=n_slots, row_stride=Lb,
                         rows_gen_stride=n_slots * Lb, rec_row_stride=Lb, rec_gen_stride=emax * Lb, G=G)
    assert (st_h.numpy() == 0).all() and (nrec_h.numpy() == e).all()
    rec = rec_h.numpy().reshape(G, emax, Lb)
    ri = ridx_h.numpy().view(np.uint16).reshape(G, emax)
    for g in sorted({0, per - 1, per, 2 * per - 1, 2 * per, G - 1} | set(rng.integers(0, G, 10).tolist())):
        st, sol, mask = oracle.decode(k, idx[g], rows[g])
        assert st == 0
        erased = np.nonzero(mask == 0)[0]
        assert list(ri[g, :e]) == list(erased)
        assert (rec[g, :e] == sol[erased]).all()
    for g in range(G):   # every generation recovers the original bytes
        assert (rec[g, :e] == src_np[g, ri[g, :e]]).all()
