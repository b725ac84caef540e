// qf_objects16.hip -- GF(2^16) Encoder16 / Decoder16 objects of the C ABI
// (decoder.rs:10-88, 536-656), the per-connection codec of Extreme mode.
// Host logic over the batch kernels of qf_gf16.hip (one generation per
// call); payload state lives in HBM.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <vector>

#include "qf_fec.h"
#include "qf_internal.h"


namespace {

constexpr uint32_t kMaxK16 = 4096;  // Extreme windows (adaptive.rs:131)

uint32_t round16(uint32_t x) { return (x + 15) & ~15u; }

// host log / exp of GF(2^16) mod 0x1100B, generator 2
struct Gf16Host {
    std::vector<uint16_t> lg, ex;
    Gf16Host() : lg(65536, 0), ex(65535) {
        uint32_t x = 1;
        for (uint32_t i = 0; i < 65535; ++i) {
            ex[i] = (uint16_t)x;
            lg[x] = (uint16_t)i;
            x <<= 1;
            if (x & 0x10000u) x ^= 0x1100Bu;
        }
    }
    uint16_t inv(uint16_t a) const { return ex[(65535 - lg[a]) % 65535]; }  // a != 0
};

const Gf16Host& gf16h() {
    static Gf16Host g;
    return g;
}

int grow(uint8_t** p, size_t* cap, size_t bytes) {
    if (bytes <= *cap) return QF_OK;
    if (*p) hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipMalloc(p, bytes) != hipSuccess) return QF_ENOMEM;
    *cap = bytes;
    return QF_OK;
}

}  // namespace

struct qf_encoder16 {
    qf_ctx* ctx = nullptr;
    uint32_t k = 0, n = 0, max_len = 0, stride = 0;
    uint8_t* d_ring = nullptr;  // k slots of `stride` bytes (zero padded)
    uint8_t* d_out = nullptr;   // repair rows
    uint8_t* d_coef = nullptr;  // big-endian coefficient blocks
    size_t out_cap = 0, coef_cap = 0;
    std::vector<uint32_t> lens;
    std::vector<uint64_t> ids;
    uint32_t count = 0, head = 0;
    std::vector<uint8_t> stage;
};

struct qf_decoder16 {
    qf_ctx* ctx = nullptr;
    uint32_t k = 0, max_len = 0, stride = 0;
    bool decoded = false, drained = false;
    // the first k rows, arrival order (decoder.rs:563-566)
    uint8_t* rows = nullptr;      // k * stride, pinned: each row is uploaded as it arrives
    std::vector<uint32_t> lens;
    std::vector<uint16_t> index;    // source column (systematic) or k (repair)
    std::vector<uint16_t> coeffs;   // k * k, repair rows (from the big-endian block)
    std::vector<uint8_t> repair;    // slot is a repair row
    uint32_t accepted = 0;
    std::vector<uint8_t> out;       // decoded sources, index order
    std::vector<uint32_t> out_len;
    uint8_t *d_rows = nullptr, *d_rec = nullptr;
    uint16_t *d_index = nullptr, *d_coeffs = nullptr, *d_rec_index = nullptr;
    uint32_t* d_nrec = nullptr;
    int32_t* d_status = nullptr;
    uint8_t* h_rec = nullptr;       // pinned download of the recovered rows (grown)
    size_t h_rec_bytes = 0;
};

extern "C" {

int qf_encoder16_new(qf_ctx* ctx, uint32_t k, uint32_t n, uint32_t max_len, qf_encoder16** out) {
    if (!ctx || !out || k == 0 || k > kMaxK16 || n < k || max_len == 0) return QF_EINVAL;
    qf_encoder16* e = new qf_encoder16();
    e->ctx = ctx;
    e->k = k;
    e->n = n;
    e->max_len = max_len;
    e->stride = round16(max_len);
    e->lens.assign(k, 0);
    e->ids.assign(k, 0);
    e->stage.assign(e->stride, 0);
    if (hipMalloc(&e->d_ring, (size_t)k * e->stride) != hipSuccess ||
        hipMemset(e->d_ring, 0, (size_t)k * e->stride) != hipSuccess) {
        qf_encoder16_free(e);
        return QF_ENOMEM;
    }
    *out = e;
    return QF_OK;
}

int qf_encoder16_free(qf_encoder16* e) {
    if (!e) return QF_OK;
    hipFree(e->d_ring);
    hipFree(e->d_out);
    hipFree(e->d_coef);
    delete e;
    return QF_OK;
}

int qf_encoder16_window_len(const qf_encoder16* e) { return e ? (int)e->count : QF_EINVAL; }

// decoder.rs:25-30: a full window drops its oldest packet
int qf_encoder16_add_source_packet(qf_encoder16* e, uint64_t id, const uint8_t* data, uint32_t len) {
    if (!e || (len && !data) || len > e->max_len) return QF_EINVAL;
    memset(e->stage.data(), 0, e->stride);
    if (len) memcpy(e->stage.data(), data, len);
    const uint32_t slot = e->head;
    hipStream_t st = (hipStream_t)qf_ctx_stream(e->ctx);
    QF_CHECK_HIP(hipMemcpyAsync(e->d_ring + (size_t)slot * e->stride, e->stage.data(), e->stride,
                                hipMemcpyHostToDevice, st));
    QF_CHECK_HIP(hipStreamSynchronize(st));
    e->lens[slot] = len;
    e->ids[slot] = id;
    e->head = (e->head + 1) % e->k;
    if (e->count < e->k) e->count++;
    return QF_OK;
}

// decoder.rs:33-75 for repairs first..first+count-1 in one launch.  Symbols are
// byte pairs: with an odd packet length the last repair byte stays 0
// (the reference's `while j + 1 < packet_len`).
int qf_encoder16_generate_repairs(qf_encoder16* e, uint32_t first, uint32_t count, uint8_t* out_data,
                                  uint32_t out_stride, uint32_t* out_len, uint8_t* out_coeffs, uint64_t* out_ids) {
    if (!e || count == 0) return QF_EINVAL;
    if (e->count < e->k) return QF_ENOTREADY;  // decoder.rs:38-40 (None)
    const uint32_t k = e->k;
    if ((uint64_t)k + first + count > 65536) return QF_ERANGE;  // gf16_inv(0)
    const uint32_t oldest = e->head;
    const uint32_t L = e->lens[oldest];  // packet_len = window[0].len
    const uint32_t newest = (e->head + k - 1) % k;
    if (out_data && out_stride < L) return QF_ETOOSMALL;
    hipStream_t st = (hipStream_t)qf_ctx_stream(e->ctx);
    const uint32_t Le = L & ~1u;
    int s = grow(&e->d_coef, &e->coef_cap, (size_t)count * k * 2);
    if (s) return s;
    s = grow(&e->d_out, &e->out_cap, (size_t)count * e->stride);
    if (s) return s;
    qf_encode_shape sh{};
    sh.k = k;
    sh.r = count;
    sh.L = Le ? Le : 2;  // L < 2: no symbols; the launch still writes the coefficient blocks
    sh.src_row_stride = e->stride;
    sh.src_gen_stride = (uint64_t)k * e->stride;
    sh.rep_row_stride = e->stride;
    sh.rep_gen_stride = (uint64_t)count * e->stride;
    s = qf::encode16_window(e->ctx, &sh, 1, e->d_ring, e->d_out, nullptr, first, oldest, e->d_coef);
    if (s != QF_OK) return s;
    if (out_data && L) {
        QF_CHECK_HIP(hipMemcpy2DAsync(out_data, out_stride, e->d_out, e->stride, Le ? Le : 1, count,
                                      hipMemcpyDeviceToHost, st));
    }
    if (out_coeffs)
        QF_CHECK_HIP(hipMemcpyAsync(out_coeffs, e->d_coef, (size_t)count * k * 2, hipMemcpyDeviceToHost, st));
    QF_CHECK_HIP(hipStreamSynchronize(st));
    for (uint32_t q = 0; q < count; ++q) {
        if (out_data && L != Le) out_data[(size_t)q * out_stride + L - 1] = 0;
        if (out_len) out_len[q] = L;
        if (out_ids) out_ids[q] = e->ids[newest] + 1 + first + q;  // decoder.rs:68
    }
    return QF_OK;
}

int qf_encoder16_generate_repair_packet(qf_encoder16* e, uint32_t j, uint8_t* out_data, uint32_t out_cap,
                                        uint32_t* out_len, uint8_t* out_coeffs, uint64_t* out_id) {
    if (!e) return QF_EINVAL;
    if (e->count < e->k) return QF_ENOTREADY;
    if (out_data && out_cap < e->lens[e->head]) return QF_ETOOSMALL;
    return qf_encoder16_generate_repairs(e, j, 1, out_data, out_cap, out_len, out_coeffs, out_id);
}

int qf_decoder16_new(qf_ctx* ctx, uint32_t k, uint32_t max_len, qf_decoder16** out) {
    if (!ctx || !out || k == 0 || k > kMaxK16 || max_len == 0) return QF_EINVAL;
    qf_decoder16* d = new qf_decoder16();
    d->ctx = ctx;
    d->k = k;
    d->max_len = max_len;
    d->stride = round16(max_len);
    d->lens.assign(k, 0);
    d->index.assign(k, 0);
    d->coeffs.assign((size_t)k * k, 0);
    d->repair.assign(k, 0);
    const bool ok = hipMalloc(&d->d_rows, (size_t)k * d->stride) == hipSuccess &&
                    hipMalloc(&d->d_rec, (size_t)k * d->stride) == hipSuccess &&
                    hipMalloc(&d->d_index, (size_t)k * 2) == hipSuccess &&
                    hipMalloc(&d->d_coeffs, (size_t)k * k * 2) == hipSuccess &&
                    hipMalloc(&d->d_rec_index, (size_t)k * 2) == hipSuccess &&
                    hipMalloc(&d->d_nrec, 4) == hipSuccess && hipMalloc(&d->d_status, 4) == hipSuccess &&
                    hipHostMalloc(reinterpret_cast<void**>(&d->rows), (size_t)k * d->stride) == hipSuccess;
    if (!ok) {
        qf_decoder16_free(d);
        return QF_ENOMEM;
    }
    *out = d;
    return QF_OK;
}

int qf_decoder16_free(qf_decoder16* d) {
    if (!d) return QF_OK;
    hipFree(d->d_rows);
    hipFree(d->d_rec);
    hipFree(d->d_index);
    hipFree(d->d_coeffs);
    hipFree(d->d_rec_index);
    hipFree(d->d_nrec);
    hipFree(d->d_status);
    if (d->rows) {
        hipStreamSynchronize((hipStream_t)qf_ctx_stream(d->ctx));  // row uploads in flight
        hipHostFree(d->rows);
    }
    if (d->h_rec) hipHostFree(d->h_rec);
    delete d;
    return QF_OK;
}

int qf_decoder16_is_decoded(const qf_decoder16* d) { return d ? (d->decoded ? 1 : 0) : QF_EINVAL; }

// decoder.rs:594-640 on the device.  Repair rows that are Cauchy rows of this
// k (c_i = gf16_inv(i ^ y), y >= k: what Encoder16 emits for an aligned
// window) go to the closed-form inverse by their y; any other row makes the
// whole system explicit (Gauss-Jordan).
static int decoder16_try_decode(qf_decoder16* d) {
    const uint32_t k = d->k;
    const auto& f = gf16h();
    uint32_t L = 0;
    for (uint32_t q = 0; q < k; ++q) L = d->lens[q] > L ? d->lens[q] : L;
    const uint32_t Le = L & ~1u;
    std::vector<uint16_t> idx(d->index);
    bool cauchy = true;
    for (uint32_t q = 0; q < k && cauchy; ++q) {
        if (!d->repair[q]) continue;
        const uint16_t* c = &d->coeffs[(size_t)q * k];
        if (!c[0]) {
            cauchy = false;
            break;
        }
        const uint32_t y = f.inv(c[0]);
        if (y < k) {
            cauchy = false;
            break;
        }
        for (uint32_t i = 0; i < k && cauchy; ++i) cauchy = c[i] == f.inv((uint16_t)(i ^ y));
        idx[q] = (uint16_t)y;
    }
    if (!cauchy)
        for (uint32_t q = 0; q < k; ++q)
            if (d->repair[q]) idx[q] = (uint16_t)k;
    hipStream_t st = (hipStream_t)qf_ctx_stream(d->ctx);
    // the rows are on the device already (uploaded as they arrived)
    QF_CHECK_HIP(hipMemcpyAsync(d->d_index, idx.data(), (size_t)k * 2, hipMemcpyHostToDevice, st));
    if (!cauchy)
        QF_CHECK_HIP(hipMemcpyAsync(d->d_coeffs, d->coeffs.data(), (size_t)k * k * 2, hipMemcpyHostToDevice, st));
    qf_decode_shape sh{};
    sh.k = k;
    sh.r = k;  // up to k erasures
    sh.L = Le ? Le : 2;
    sh.max_rows = k;
    sh.row_stride = d->stride;
    sh.rows_gen_stride = (uint64_t)k * d->stride;
    sh.rec_row_stride = d->stride;
    sh.rec_gen_stride = (uint64_t)k * d->stride;
    int s = qf_decode16_batch(d->ctx, &sh, 1, d->d_rows, d->d_index, nullptr, cauchy ? nullptr : d->d_coeffs,
                              d->d_rec, d->d_rec_index, d->d_nrec, d->d_status);
    if (s != QF_OK) return s;
    int32_t status = 0;
    uint32_t nrec = 0;
    QF_CHECK_HIP(hipMemcpyAsync(&status, d->d_status, 4, hipMemcpyDeviceToHost, st));
    QF_CHECK_HIP(hipMemcpyAsync(&nrec, d->d_nrec, 4, hipMemcpyDeviceToHost, st));
    QF_CHECK_HIP(hipStreamSynchronize(st));
    if (status != QF_OK) return status;  // singular: try_decode -> false (decoder.rs:604-606)
    std::vector<uint16_t> ridx(nrec);
    if (nrec) {
        const size_t need = (size_t)nrec * d->stride;
        if (need > d->h_rec_bytes) {
            if (d->h_rec) hipHostFree(d->h_rec);
            d->h_rec = nullptr;
            d->h_rec_bytes = 0;
            if (hipHostMalloc(reinterpret_cast<void**>(&d->h_rec), need) != hipSuccess) return QF_ENOMEM;
            d->h_rec_bytes = need;
        }
        QF_CHECK_HIP(hipMemcpyAsync(ridx.data(), d->d_rec_index, (size_t)nrec * 2, hipMemcpyDeviceToHost, st));
        QF_CHECK_HIP(hipMemcpyAsync(d->h_rec, d->d_rec, need, hipMemcpyDeviceToHost, st));
        QF_CHECK_HIP(hipStreamSynchronize(st));
    }
    const uint8_t* rec = d->h_rec;
    d->out.assign((size_t)k * d->stride, 0);
    d->out_len.assign(k, 0);
    for (uint32_t q = 0; q < k; ++q)
        if (!d->repair[q]) {
            const uint32_t i = d->index[q];
            memcpy(&d->out[(size_t)i * d->stride], &d->rows[(size_t)q * d->stride], d->stride);
            d->out_len[i] = d->lens[q];
        }
    for (uint32_t m = 0; m < nrec; ++m) {
        const uint32_t i = ridx[m];
        memcpy(&d->out[(size_t)i * d->stride], rec + (size_t)m * d->stride, Le);
        d->out_len[i] = L;  // an odd length's last byte carries no symbol: 0
    }
    d->decoded = true;
    return QF_OK;
}

// decoder.rs:555-592
int qf_decoder16_add_packet(qf_decoder16* d, uint64_t id, int is_systematic, const uint8_t* data, uint32_t len,
                            const uint8_t* coeffs, uint32_t coeff_len) {
    if (!d || (len && !data) || len > d->max_len) return QF_EINVAL;
    if (d->decoded || d->accepted >= d->k) return d->decoded ? 1 : 0;
    const uint32_t k = d->k, q = d->accepted;
    uint16_t* row = &d->coeffs[(size_t)q * k];
    memset(row, 0, (size_t)k * 2);
    if (is_systematic) {
        d->index[q] = (uint16_t)(id % k);  // decoder.rs:561-566, duplicates not filtered
        d->repair[q] = 0;
    } else {
        if (!coeffs) return QF_EINVAL;  // Err("missing coeffs")
        for (uint32_t i = 0; i < k && 2 * i + 1 < coeff_len; ++i)
            row[i] = (uint16_t)(coeffs[2 * i] << 8 | coeffs[2 * i + 1]);  // decoder.rs:568-573
        d->index[q] = (uint16_t)k;
        d->repair[q] = 1;
    }
    memset(&d->rows[(size_t)q * d->stride], 0, d->stride);
    if (len) memcpy(&d->rows[(size_t)q * d->stride], data, len);
    // to the device now; rows is pinned and slot q is not rewritten while
    // this decoder lives, so the copy needs no wait
    QF_CHECK_HIP(hipMemcpyAsync(d->d_rows + (size_t)q * d->stride, &d->rows[(size_t)q * d->stride], d->stride,
                                hipMemcpyHostToDevice, (hipStream_t)qf_ctx_stream(d->ctx)));
    d->lens[q] = len;
    d->accepted++;
    if (d->accepted == k) {
        int s = decoder16_try_decode(d);
        if (s == QF_ERANK) return 0;
        if (s != QF_OK) return s;
    }
    return d->decoded ? 1 : 0;
}

// decoder.rs:643-655, returning the whole generation in index order (as the
// GF(2^8) decoder, decoder.rs:785-790)
int qf_decoder16_get_decoded_packets(qf_decoder16* d, uint8_t* out_data, uint32_t out_stride, uint32_t* out_len,
                                     uint64_t* out_ids, uint32_t* count) {
    if (!d || !count) return QF_EINVAL;
    *count = 0;
    if (!d->decoded || d->drained) return QF_OK;
    uint32_t need = 0;
    for (uint32_t i = 0; i < d->k; ++i) need = d->out_len[i] > need ? d->out_len[i] : need;
    if (out_data && out_stride < need) return QF_ETOOSMALL;
    for (uint32_t i = 0; i < d->k; ++i) {
        if (out_data) memcpy(out_data + (size_t)i * out_stride, &d->out[(size_t)i * d->stride], d->out_len[i]);
        if (out_len) out_len[i] = d->out_len[i];
        if (out_ids) out_ids[i] = i;
    }
    *count = d->k;
    d->drained = true;
    return QF_OK;
}

}  // extern "C"
