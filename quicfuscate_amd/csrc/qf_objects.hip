// qf_objects.hip -- per-connection Encoder / Decoder objects of the C ABI,
// mirroring the reference's Rust API call for call (decoder.rs:155-299,
// 658-791).  Payload state lives in HBM; each call is one batch launch of
// the same kernels the batch API uses (G = 1 generation).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "gf256_tables.h"
#include "qf_fec.h"
#include "qf_bs.h"
#include "qf_internal.h"

#define QF_CHECK_HIP(expr)                         \
    do {                                           \
        hipError_t _e = (expr);                    \
        if (_e != hipSuccess) return QF_EDEVICE;   \
    } while (0)

static inline uint32_t round16(uint32_t x) { return (x + 15) & ~15u; }

struct qf_encoder {
    qf_ctx* ctx = nullptr;
    uint32_t k = 0, n = 0, max_len = 0, stride = 0;
    // 2k slots of `stride` bytes (zero padded): packet c sits in slots c % k
    // and c % k + k, so the window (oldest first) is always the k contiguous
    // slots from `head` -- a plain batch encode with the cached Cauchy matrix
    uint8_t* d_ring = nullptr;
    uint8_t* d_out = nullptr;   // up to 256 repair rows
    std::vector<uint32_t> lens;
    std::vector<uint64_t> ids;
    uint32_t count = 0;  // packets in the window (<= k)
    uint32_t head = 0;   // next slot to write (== oldest slot once full)
    uint8_t* h_stage = nullptr;      // pinned staging of one packet
    hipEvent_t stage_done = nullptr; // its copies have landed
    std::vector<uint8_t> win;        // Cauchy rows 0..r-1 in window order (cached)
    // small-batch kernel (QF_ENCODE_SMALL != 0): it reads the ring rotated,
    // so each packet is uploaded once; otherwise the double ring keeps the
    // window contiguous for the bit-sliced kernels
    bool ring_rot = true;
    uint8_t* h_out = nullptr;        // pinned download of the repair rows
    size_t h_out_bytes = 0;
};

struct qf_decoder {
    qf_ctx* ctx = nullptr;
    uint32_t k = 0, max_len = 0, stride = 0;
    bool decoded = false, drained = false;
    // accepted rows, in arrival order (the first k win)
    uint8_t* rows = nullptr;     // k * stride, pinned: each row is uploaded as it arrives
    std::vector<uint32_t> lens;    // k
    std::vector<uint16_t> index;   // k: source index (< k) or k (repair)
    std::vector<uint8_t> coeffs;   // k * k (repair rows)
    std::vector<int32_t> sys_slot; // per source index: accepted slot or -1
    std::vector<uint64_t> sys_id;  // per source index: the received packet's own id
    uint32_t accepted = 0;
    // decoded output, source index order
    std::vector<uint8_t> out;      // k * stride
    std::vector<uint32_t> out_len;
    // device buffers for one generation
    uint8_t* d_rows = nullptr;
    uint8_t* d_coeffs = nullptr;
    uint16_t* d_index = nullptr;
    uint8_t* d_rec = nullptr;
    uint16_t* d_rec_index = nullptr;
    uint32_t* d_nrec = nullptr;
    int32_t* d_status = nullptr;
    uint8_t* h_rec = nullptr;       // pinned download of the recovered rows
};

extern "C" {

int qf_encoder_new(qf_ctx* ctx, uint32_t k, uint32_t n, uint32_t max_len, qf_encoder** out) {
    if (!ctx || !out || k == 0 || k > 256 || n < k || max_len == 0) return QF_EINVAL;
    qf_encoder* e = new qf_encoder();
    e->ctx = ctx;
    e->k = k;
    e->n = n;
    e->max_len = max_len;
    e->stride = round16(max_len);
    e->lens.assign(k, 0);
    e->ids.assign(k, 0);
    e->ring_rot = qf::small_encode_enabled();
    if (hipMalloc(&e->d_ring, (size_t)2 * k * e->stride) != hipSuccess ||
        hipMalloc(&e->d_out, (size_t)256 * e->stride) != hipSuccess ||
        hipMemset(e->d_ring, 0, (size_t)2 * k * e->stride) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&e->h_stage), e->stride) != hipSuccess ||
        hipEventCreateWithFlags(&e->stage_done, hipEventDisableTiming) != hipSuccess) {
        qf_encoder_free(e);
        return QF_ENOMEM;
    }
    *out = e;
    return QF_OK;
}

int qf_encoder_free(qf_encoder* e) {
    if (!e) return QF_OK;
    if (e->stage_done) {
        hipEventSynchronize(e->stage_done);
        hipEventDestroy(e->stage_done);
    }
    if (e->h_stage) hipHostFree(e->h_stage);
    if (e->h_out) hipHostFree(e->h_out);
    if (e->d_ring) hipFree(e->d_ring);
    if (e->d_out) hipFree(e->d_out);
    delete e;
    return QF_OK;
}

int qf_encoder_window_len(const qf_encoder* e) { return e ? (int)e->count : QF_EINVAL; }

// decoder.rs:164-169: when the window holds k packets the oldest is dropped.
int qf_encoder_add_source_packet(qf_encoder* e, uint64_t id, const uint8_t* data, uint32_t len) {
    if (!e || (len && !data) || len > e->max_len) return QF_EINVAL;
    // the staging buffer is reused: the previous packet's copies must have landed
    QF_CHECK_HIP(hipEventSynchronize(e->stage_done));
    memset(e->h_stage, 0, e->stride);
    if (len) memcpy(e->h_stage, data, len);
    const uint32_t slot = e->head;
    hipStream_t st = (hipStream_t)qf_ctx_stream(e->ctx);
    QF_CHECK_HIP(hipMemcpyAsync(e->d_ring + (size_t)slot * e->stride, e->h_stage, e->stride,
                                hipMemcpyHostToDevice, st));
    if (!e->ring_rot)
        QF_CHECK_HIP(hipMemcpyAsync(e->d_ring + (size_t)(slot + e->k) * e->stride, e->h_stage, e->stride,
                                    hipMemcpyHostToDevice, st));
    QF_CHECK_HIP(hipEventRecord(e->stage_done, st));
    e->lens[slot] = len;
    e->ids[slot] = id;
    e->head = (e->head + 1) % e->k;
    if (e->count < e->k) e->count++;
    return QF_OK;
}

int qf_encoder_generate_repairs(qf_encoder* e, uint32_t first, uint32_t count, uint8_t* out_data,
                                uint32_t out_stride, uint32_t* out_len, uint8_t* out_coeffs,
                                uint64_t* out_ids) {
    if (!e || count == 0 || count > 256) return QF_EINVAL;
    if (e->count < e->k) return QF_ENOTREADY;  // decoder.rs:177-179 (None)
    const uint32_t k = e->k;
    const uint32_t oldest = e->head;  // window full: head is the oldest slot
    const uint32_t L = e->lens[oldest];  // packet_len = window[0].len
    const uint32_t newest = (e->head + k - 1) % k;
    if (out_data && out_stride < L) return QF_ETOOSMALL;
    // Cauchy rows first..first+count-1 in window order (decoder.rs:280-298),
    // computed once per encoder
    if ((uint64_t)k + first + count > 256) return QF_ERANGE;  // gf_inv(0)
    const uint32_t rows = first + count;
    if (e->win.size() < (size_t)rows * k) {
        const auto& f = qf::gf();
        e->win.resize((size_t)rows * k);
        for (uint32_t q = 0; q < rows; ++q)
            for (uint32_t i = 0; i < k; ++i)
                if (!f.inv((uint8_t)((uint8_t)i ^ (uint8_t)(k + q)), &e->win[(size_t)q * k + i])) return QF_ERANGE;
    }
    const uint8_t* win = e->win.data() + (size_t)first * k;
    if (L > 0) {
        // the window is contiguous in the double ring: repairs 0..count-1 are
        // the cached Cauchy code (k, count) (generated kernel or cached
        // tables); a later first row goes through explicit coefficients
        int s;
        if (e->ring_rot) {
            s = qf::encode_ring_window(e->ctx, k, first, count, L, e->d_ring, e->stride, oldest, e->d_out,
                                       e->stride);
        } else {
            qf_encode_shape sh{};
            sh.k = k;
            sh.r = count;
            sh.L = L;
            sh.src_row_stride = e->stride;
            sh.src_gen_stride = (uint64_t)k * e->stride;
            sh.rep_row_stride = e->stride;
            sh.rep_gen_stride = (uint64_t)count * e->stride;
            s = qf_encode_batch(e->ctx, &sh, 1, e->d_ring + (size_t)oldest * e->stride, e->d_out,
                                first == 0 ? nullptr : win);
        }
        if (s != QF_OK) return s;
        hipStream_t st = (hipStream_t)qf_ctx_stream(e->ctx);
        if (out_data) {
            // one contiguous D2H into pinned memory (a copy into the caller's
            // pageable rows would go through the runtime's staging), then
            // the rows out on the host
            const size_t bytes = (size_t)count * e->stride;
            if (e->h_out_bytes < bytes) {
                QF_CHECK_HIP(hipStreamSynchronize(st));
                if (e->h_out) hipHostFree(e->h_out);
                e->h_out = nullptr;
                e->h_out_bytes = 0;
                if (hipHostMalloc(reinterpret_cast<void**>(&e->h_out), (size_t)256 * e->stride) != hipSuccess)
                    return QF_ENOMEM;
                e->h_out_bytes = (size_t)256 * e->stride;
            }
            QF_CHECK_HIP(hipMemcpyAsync(e->h_out, e->d_out, bytes, hipMemcpyDeviceToHost, st));
            QF_CHECK_HIP(hipStreamSynchronize(st));
            for (uint32_t q = 0; q < count; ++q)
                memcpy(out_data + (size_t)q * out_stride, e->h_out + (size_t)q * e->stride, L);
        } else {
            QF_CHECK_HIP(hipStreamSynchronize(st));
        }
    }
    for (uint32_t q = 0; q < count; ++q) {
        if (out_len) out_len[q] = L;
        if (out_ids) out_ids[q] = e->ids[newest] + 1 + first + q;  // decoder.rs:267
        if (out_coeffs) memcpy(out_coeffs + (size_t)q * k, win + (size_t)q * k, k);
    }
    return QF_OK;
}

int qf_encoder_generate_repair_packet(qf_encoder* e, uint32_t j, uint8_t* out_data, uint32_t out_cap,
                                      uint32_t* out_len, uint8_t* out_coeffs, uint64_t* out_id) {
    if (!e) return QF_EINVAL;
    if (e->count < e->k) return QF_ENOTREADY;
    const uint32_t L = e->lens[e->head];
    if (out_data && out_cap < L) return QF_ETOOSMALL;
    return qf_encoder_generate_repairs(e, j, 1, out_data, out_cap, out_len, out_coeffs, out_id);
}

int qf_decoder_new(qf_ctx* ctx, uint32_t k, uint32_t max_len, qf_decoder** out) {
    if (!ctx || !out || k == 0 || k > 256 || max_len == 0) return QF_EINVAL;
    qf_decoder* d = new qf_decoder();
    d->ctx = ctx;
    d->k = k;
    d->max_len = max_len;
    d->stride = round16(max_len);
    d->lens.assign(k, 0);
    d->index.assign(k, 0);
    d->coeffs.assign((size_t)k * k, 0);
    d->sys_slot.assign(k, -1);
    d->sys_id.assign(k, 0);
    const uint32_t emax = k < 128 ? k : 128;
    bool ok = hipMalloc(&d->d_rows, (size_t)k * d->stride) == hipSuccess &&
              hipMalloc(&d->d_coeffs, (size_t)k * k) == hipSuccess &&
              hipMalloc(&d->d_index, (size_t)k * 2) == hipSuccess &&
              hipMalloc(&d->d_rec, (size_t)emax * d->stride) == hipSuccess &&
              hipMalloc(&d->d_rec_index, (size_t)emax * 2) == hipSuccess &&
              hipMalloc(&d->d_nrec, 4) == hipSuccess && hipMalloc(&d->d_status, 4) == hipSuccess &&
              hipHostMalloc(reinterpret_cast<void**>(&d->rows), (size_t)k * d->stride) == hipSuccess &&
              hipHostMalloc(reinterpret_cast<void**>(&d->h_rec), (size_t)emax * d->stride) == hipSuccess;
    if (!ok) {
        qf_decoder_free(d);
        return QF_ENOMEM;
    }
    *out = d;
    return QF_OK;
}

int qf_decoder_free(qf_decoder* d) {
    if (!d) return QF_OK;
    hipFree(d->d_rows);
    hipFree(d->d_coeffs);
    hipFree(d->d_index);
    hipFree(d->d_rec);
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

int qf_decoder_is_decoded(const qf_decoder* d) { return d ? (d->decoded ? 1 : 0) : QF_EINVAL; }

// decoder.rs:704-783 for the k accepted rows, on the device.
static int decoder_try_decode(qf_decoder* d) {
    const uint32_t k = d->k;
    uint32_t L = 0;
    for (uint32_t q = 0; q < k; ++q) L = d->lens[q] > L ? d->lens[q] : L;
    if (L == 0) L = 1;
    hipStream_t st = (hipStream_t)qf_ctx_stream(d->ctx);
    const uint32_t emax = k < 128 ? k : 128;
    // Repair rows that are Cauchy rows of this k (c_i = gf_inv(i ^ y), y =
    // k + j: what Encoder emits for a window aligned with the generation)
    // decode by their repair index on the Cauchy paths (generated kernels);
    // any other row keeps the whole system explicit.
    const auto& f = qf::gf();
    std::vector<uint16_t> idx(d->index);
    uint32_t rmax = 0;
    bool cauchy = true;
    for (uint32_t q = 0; q < k && cauchy; ++q) {
        if (d->index[q] != k) continue;  // systematic
        const uint8_t* c = &d->coeffs[(size_t)q * k];
        uint8_t y = 0;
        if (!f.inv(c[0], &y) || y < k) {   // c_0 = gf_inv(y)
            cauchy = false;
            break;
        }
        for (uint32_t i = 0; i < k && cauchy; ++i) {
            uint8_t v = 0;
            cauchy = f.inv((uint8_t)(i ^ y), &v) && v == c[i];
        }
        idx[q] = y;
        rmax = std::max<uint32_t>(rmax, (uint32_t)y - k + 1);
    }
    cauchy = cauchy && rmax <= emax;
    if (!cauchy) {
        idx = d->index;
        QF_CHECK_HIP(hipMemcpyAsync(d->d_coeffs, d->coeffs.data(), (size_t)k * k, hipMemcpyHostToDevice, st));
    }
    // the rows are on the device already (uploaded as they arrived)
    QF_CHECK_HIP(hipMemcpyAsync(d->d_index, idx.data(), (size_t)k * 2, hipMemcpyHostToDevice, st));
    qf_decode_shape sh{};
    sh.k = k;
    uint32_t rc = std::max<uint32_t>(rmax, 1);
    if (cauchy) {
        // the Cauchy code of (k, r') holds rows 0..r'-1: take the smallest r'
        // >= rmax with generated kernels, so the decode runs on them
        for (uint32_t r2 = rc; r2 <= emax && k + r2 <= 256; ++r2)
            if (qf::syn_available(k, r2) || qf::bs_available(k, r2)) {
                rc = r2;
                break;
            }
    }
    sh.r = cauchy ? rc : emax;
    sh.L = L;
    sh.max_rows = k;
    sh.row_stride = d->stride;
    sh.rows_gen_stride = (uint64_t)k * d->stride;
    sh.rec_row_stride = d->stride;
    sh.rec_gen_stride = (uint64_t)emax * d->stride;
    int s = qf_decode_batch(d->ctx, &sh, 1, d->d_rows, d->d_index, nullptr, cauchy ? nullptr : d->d_coeffs,
                            d->d_rec, d->d_rec_index, d->d_nrec, d->d_status);
    if (s != QF_OK) return s;
    int32_t status = 0;
    uint32_t nrec = 0;
    QF_CHECK_HIP(hipMemcpyAsync(&status, d->d_status, 4, hipMemcpyDeviceToHost, st));
    QF_CHECK_HIP(hipMemcpyAsync(&nrec, d->d_nrec, 4, hipMemcpyDeviceToHost, st));
    QF_CHECK_HIP(hipStreamSynchronize(st));
    if (status != QF_OK) return status;  // singular: stays undecoded (decoder.rs:756-758)
    std::vector<uint16_t> ridx(nrec);
    const uint8_t* rec = d->h_rec;
    if (nrec) {
        QF_CHECK_HIP(hipMemcpyAsync(ridx.data(), d->d_rec_index, (size_t)nrec * 2, hipMemcpyDeviceToHost, st));
        QF_CHECK_HIP(hipMemcpyAsync(d->h_rec, d->d_rec, (size_t)nrec * d->stride, hipMemcpyDeviceToHost, st));
        QF_CHECK_HIP(hipStreamSynchronize(st));
    }
    d->out.assign((size_t)k * d->stride, 0);
    d->out_len.assign(k, 0);
    for (uint32_t i = 0; i < k; ++i) {
        const int32_t q = d->sys_slot[i];
        if (q >= 0) {
            memcpy(&d->out[(size_t)i * d->stride], &d->rows[(size_t)q * d->stride], d->stride);
            d->out_len[i] = d->lens[q];
        }
    }
    for (uint32_t m = 0; m < nrec; ++m) {
        const uint32_t i = ridx[m];
        memcpy(&d->out[(size_t)i * d->stride], rec + (size_t)m * d->stride, L);
        d->out_len[i] = L;
    }
    d->decoded = true;
    return QF_OK;
}

int qf_decoder_add_packet(qf_decoder* d, uint64_t id, int is_systematic, const uint8_t* data,
                          uint32_t len, const uint8_t* coeffs, uint32_t coeff_len) {
    if (!d || (len && !data)) return QF_EINVAL;
    if (len > d->max_len) return QF_EINVAL;
    // decoder.rs:679-681
    if (d->decoded || d->accepted >= d->k) return d->decoded ? 1 : 0;
    const uint32_t k = d->k;
    const uint32_t q = d->accepted;
    if (is_systematic) {
        const uint32_t idx = (uint32_t)(id % k);  // decoder.rs:684
        if (d->sys_slot[idx] >= 0) return d->decoded ? 1 : 0;  // duplicate (687-691)
        d->sys_slot[idx] = (int32_t)q;
        d->sys_id[idx] = id;  // systematic_packets[index] = Some(packet) keeps packet.id (decoder.rs:688)
        d->index[q] = (uint16_t)idx;
        memset(&d->coeffs[(size_t)q * k], 0, k);
    } else {
        if (!coeffs) return QF_EINVAL;  // "Repair packet missing coefficients."
        d->index[q] = (uint16_t)k;
        memset(&d->coeffs[(size_t)q * k], 0, k);
        memcpy(&d->coeffs[(size_t)q * k], coeffs, coeff_len < k ? coeff_len : k);
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
        int s = decoder_try_decode(d);
        if (s == QF_ERANK) return 0;
        if (s != QF_OK) return s;
    }
    return d->decoded ? 1 : 0;
}

int qf_decoder_get_decoded_packets(qf_decoder* d, uint8_t* out_data, uint32_t out_stride,
                                   uint32_t* out_len, uint64_t* out_ids, uint32_t* count) {
    if (!d || !count) return QF_EINVAL;
    *count = 0;
    if (!d->decoded || d->drained) return QF_OK;
    uint32_t need = 0;
    for (uint32_t i = 0; i < d->k; ++i) need = d->out_len[i] > need ? d->out_len[i] : need;
    if (out_data && out_stride < need) return QF_ETOOSMALL;
    for (uint32_t i = 0; i < d->k; ++i) {
        if (out_data) memcpy(out_data + (size_t)i * out_stride, &d->out[(size_t)i * d->stride], d->out_len[i]);
        if (out_len) out_len[i] = d->out_len[i];
        // a received systematic packet keeps its own id (decoder.rs:688); a
        // reconstructed one gets id = i (decoder.rs:771)
        if (out_ids) out_ids[i] = d->sys_slot[i] >= 0 ? d->sys_id[i] : i;
    }
    *count = d->k;
    d->drained = true;  // get_decoded_packets take()s the packets
    return QF_OK;
}

}  // extern "C"
