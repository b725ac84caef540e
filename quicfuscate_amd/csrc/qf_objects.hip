// qf_objects.hip -- per-connection Encoder / Decoder objects of the C ABI,
// mirroring the reference's Rust API call for call (decoder.rs:155-299,
// 658-791).  Payload state lives in HBM; each call is one batch launch of
// the same kernels the batch API uses (G = 1 generation).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <thread>
#include <unordered_map>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gf256_tables.h"
#include "qf_fec.h"
#include "qf_bs.h"
#include "qf_internal.h"
#include "qf_kernels.h"


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
    // fused per-packet send (QF_SEND_FUSED != 0, rotated ring): the packet that
    // fills the window waits in h_fresh until generate_repairs, whose one
    // kernel gets it in its arguments, writes it into its ring slot and stores
    // the repairs straight into host-coherent h_rep (no copy kernels)
    uint8_t* h_fresh = nullptr;
    uint8_t* h_rep = nullptr;        // 256 rows of `stride` bytes
    bool pending = false;
    uint32_t pend_slot = 0;
};

// decoder output block: status (4 B), count (4 B), pad, recovered indices
// (<= 128 x 2 B), then the recovered rows
constexpr size_t kOutMeta = 512;

struct qf_decoder {
    qf_ctx* ctx = nullptr;
    uint32_t k = 0, max_len = 0, stride = 0;
    bool decoded = false, drained = false;
    // a decode attempt failed on the device (not a singular system): the
    // next add on this decoder re-uploads the k rows from the pinned host
    // copy and tries again, instead of the generation staying undecodable
    bool retry = false;
    // accepted rows, in arrival order (the first k win)
    uint8_t* rows = nullptr;     // k * stride, pinned: each row is uploaded as it arrives
    std::vector<uint32_t> lens;    // k
    std::vector<uint16_t> index;   // k: source index (< k) or k (repair)
    std::vector<uint8_t> coeffs;   // k * k (repair rows)
    std::vector<int32_t> sys_slot; // per source index: accepted slot or -1
    std::vector<uint64_t> sys_id;  // per source index: the received packet's own id
    uint32_t accepted = 0;
    uint32_t uploaded = 0;         // rows [0, uploaded) are on the device
    // decoded output, source index order
    std::vector<uint8_t> out;      // k * stride
    std::vector<uint32_t> out_len;
    // device buffers for one generation.  d_rows holds the k row slots and,
    // right after them, the row-index array (d_index), so that the rows still
    // on the host and the indices go up in one copy; d_out holds status,
    // count and recovered indices (first 512 bytes) and then the recovered
    // rows, so that one copy brings all of them down (h_out mirrors it).
    uint8_t* d_rows = nullptr;
    uint8_t* d_coeffs = nullptr;
    uint16_t* d_index = nullptr;
    uint8_t* d_out = nullptr;
    uint8_t* d_rec = nullptr;
    uint16_t* d_rec_index = nullptr;
    uint32_t* d_nrec = nullptr;
    int32_t* d_status = nullptr;
    uint8_t* h_out = nullptr;       // pinned mirror of d_out
    uint8_t* h_rec = nullptr;       // h_out + kOutMeta
    uint16_t* h_index = nullptr;    // pinned, right after the host rows
    // k > 256 (Wiedemann strategy): recovered rows, grown to e rows on demand
    uint8_t* d_wrec = nullptr;
    uint32_t wrec_rows = 0;
    uint32_t w_tries = 0;           // init vectors the last Wiedemann solve used
};

namespace {

bool send_fused_enabled(qf_ctx* ctx) { return qf::ctx_opt(ctx, QF_OPT_SEND_FUSED) != 0; }

// Upload a packet still waiting for the fused send into its ring slot
// (through the staging buffer, as add_source_packet does).
int encoder_flush(qf_encoder* e) {
    if (!e->pending) return QF_OK;
    QF_CHECK_HIP(hipEventSynchronize(e->stage_done));
    memcpy(e->h_stage, e->h_fresh, e->stride);
    hipStream_t st = (hipStream_t)qf_ctx_stream(e->ctx);
    QF_CHECK_HIP(hipMemcpyAsync(e->d_ring + (size_t)e->pend_slot * e->stride, e->h_stage, e->stride,
                                hipMemcpyHostToDevice, st));
    QF_CHECK_HIP(hipEventRecord(e->stage_done, st));
    e->pending = false;
    return QF_OK;
}

// Cauchy rows 0..rows-1 in window order (decoder.rs:280-298), cached per encoder
bool window_rows(qf_encoder* e, uint32_t rows) {
    const uint32_t k = e->k;
    if (e->win.size() >= (size_t)rows * k) return true;
    const auto& f = qf::gf();
    std::vector<uint8_t> w((size_t)rows * k);
    for (uint32_t q = 0; q < rows; ++q)
        for (uint32_t i = 0; i < k; ++i)
            if (!f.inv((uint8_t)((uint8_t)i ^ (uint8_t)(k + q)), &w[(size_t)q * k + i])) return false;
    e->win.swap(w);
    return true;
}

}  // namespace

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
    e->ring_rot = qf::small_encode_enabled(ctx);
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
    if (e->h_fresh || e->h_rep) hipStreamSynchronize((hipStream_t)qf_ctx_stream(e->ctx));
    if (e->h_fresh) hipHostFree(e->h_fresh);
    if (e->h_rep) hipHostFree(e->h_rep);
    if (e->d_ring) hipFree(e->d_ring);
    if (e->d_out) hipFree(e->d_out);
    delete e;
    return QF_OK;
}

int qf_encoder_window_len(const qf_encoder* e) { return e ? (int)e->count : QF_EINVAL; }

// decoder.rs:164-169: when the window holds k packets the oldest is dropped.
int qf_encoder_add_source_packet(qf_encoder* e, uint64_t id, const uint8_t* data, uint32_t len) {
    if (!e || (len && !data) || len > e->max_len) return QF_EINVAL;
    // a packet that filled the window but was not encoded goes up first
    if (int s = encoder_flush(e)) return s;
    const uint32_t slot = e->head;
    // (the packet travels in the kernel arguments: stride <= 16 SEND_PKT_UNITS)
    if (e->ring_rot && e->count + 1 >= e->k && e->stride <= 16 * qf::SEND_PKT_UNITS && send_fused_enabled(e->ctx)) {
        // the window will be full: keep the packet for the fused send
        if (!e->h_fresh) {
            if (hipHostMalloc(reinterpret_cast<void**>(&e->h_fresh), e->stride) != hipSuccess) return QF_ENOMEM;
        }
        // (h_fresh is free: the last fused send synchronised its stream, the
        // last flush copied it out on the host)
        memset(e->h_fresh, 0, e->stride);
        if (len) memcpy(e->h_fresh, data, len);
        e->pending = true;
        e->pend_slot = slot;
        e->lens[slot] = len;
        e->ids[slot] = id;
        e->head = (e->head + 1) % e->k;
        if (e->count < e->k) e->count++;
        return QF_OK;
    }
    // the staging buffer is reused: the previous packet's copies must have landed
    QF_CHECK_HIP(hipEventSynchronize(e->stage_done));
    memset(e->h_stage, 0, e->stride);
    if (len) memcpy(e->h_stage, data, len);
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
    if (!window_rows(e, first + count)) return QF_ERANGE;
    const uint8_t* win = e->win.data() + (size_t)first * k;
    if (e->pending && L > 0 && out_data) {
        // fused send: one kernel reads the new packet from h_fresh, puts it in
        // its ring slot and writes the repairs into h_rep
        if (!e->h_rep) {
            if (hipHostMalloc(reinterpret_cast<void**>(&e->h_rep), (size_t)256 * e->stride, hipHostMallocCoherent) !=
                hipSuccess)
                return QF_ENOMEM;
        }
        int s = qf::encode_ring_window(e->ctx, k, first, count, L, e->d_ring, e->stride, oldest, e->h_rep, e->stride,
                                       e->h_fresh, e->d_ring + (size_t)e->pend_slot * e->stride, e->stride / 16);
        if (s != QF_OK) return s;
        e->pending = false;
        QF_CHECK_HIP(hipStreamSynchronize((hipStream_t)qf_ctx_stream(e->ctx)));
        for (uint32_t q = 0; q < count; ++q)
            memcpy(out_data + (size_t)q * out_stride, e->h_rep + (size_t)q * e->stride, L);
        for (uint32_t q = 0; q < count; ++q) {
            if (out_len) out_len[q] = L;
            if (out_ids) out_ids[q] = e->ids[newest] + 1 + first + q;  // decoder.rs:267
            if (out_coeffs) memcpy(out_coeffs + (size_t)q * k, win + (size_t)q * k, k);
        }
        return QF_OK;
    }
    if (int s = encoder_flush(e)) return s;
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
    if (!ctx || !out || k == 0 || k > QF_DECODER_MAX_K || max_len == 0) return QF_EINVAL;
    const bool wied = k > 256;   // decoder.rs:660-664
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
    const size_t rows_bytes = (size_t)k * d->stride + round16(2 * k);
    const size_t out_bytes = kOutMeta + (size_t)emax * d->stride;
    bool ok = hipMalloc(&d->d_rows, rows_bytes) == hipSuccess &&
              (wied || hipMalloc(&d->d_coeffs, (size_t)k * k) == hipSuccess) &&
              hipMalloc(&d->d_out, out_bytes) == hipSuccess &&
              hipHostMalloc(reinterpret_cast<void**>(&d->rows), rows_bytes) == hipSuccess &&
              hipHostMalloc(reinterpret_cast<void**>(&d->h_out), out_bytes) == hipSuccess;
    if (!ok) {
        qf_decoder_free(d);
        return QF_ENOMEM;
    }
    d->d_index = reinterpret_cast<uint16_t*>(d->d_rows + (size_t)k * d->stride);
    d->h_index = reinterpret_cast<uint16_t*>(d->rows + (size_t)k * d->stride);
    d->d_status = reinterpret_cast<int32_t*>(d->d_out);
    d->d_nrec = reinterpret_cast<uint32_t*>(d->d_out + 4);
    d->d_rec_index = reinterpret_cast<uint16_t*>(d->d_out + 16);
    d->d_rec = d->d_out + kOutMeta;
    d->h_rec = d->h_out + kOutMeta;
    *out = d;
    return QF_OK;
}

int qf_decoder_free(qf_decoder* d) {
    if (!d) return QF_OK;
    hipFree(d->d_rows);
    hipFree(d->d_coeffs);
    hipFree(d->d_out);
    hipFree(d->d_wrec);
    if (d->rows) {
        hipStreamSynchronize((hipStream_t)qf_ctx_stream(d->ctx));  // row uploads in flight
        hipHostFree(d->rows);
    }
    if (d->h_out) hipHostFree(d->h_out);
    delete d;
    return QF_OK;
}

int qf_decoder_is_decoded(const qf_decoder* d) { return d ? (d->decoded ? 1 : 0) : QF_EINVAL; }

int qf_decoder_strategy(const qf_decoder* d) {
    if (!d) return QF_EINVAL;
    return d->k > 256 ? QF_STRATEGY_WIEDEMANN : QF_STRATEGY_GAUSSIAN;
}

int qf_decoder_solve_attempts(const qf_decoder* d) {
    if (!d) return QF_EINVAL;
    return (int)d->w_tries;
}

// How the k accepted rows decode (decoder.rs:704-783): repair rows that are
// Cauchy rows of this k (c_i = gf_inv(i ^ y), y = k + j: what Encoder emits
// for a window aligned with the generation) decode by their repair index on
// the Cauchy paths (generated kernels); any other row keeps the whole system
// explicit.
struct DecPlan {
    uint32_t L = 1, rc = 1;
    bool cauchy = true;
    std::vector<uint16_t> idx;
};

static void decoder_plan(const qf_decoder* d, DecPlan* p) {
    const uint32_t k = d->k;
    uint32_t L = 0;
    for (uint32_t q = 0; q < k; ++q) L = d->lens[q] > L ? d->lens[q] : L;
    p->L = L == 0 ? 1 : L;
    const uint32_t emax = k < 128 ? k : 128;
    const auto& f = qf::gf();
    p->idx = d->index;
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
        p->idx[q] = y;
        rmax = std::max<uint32_t>(rmax, (uint32_t)y - k + 1);
    }
    p->cauchy = cauchy && rmax <= emax;
    if (!p->cauchy) p->idx = d->index;
    uint32_t rc = std::max<uint32_t>(rmax, 1);
    if (p->cauchy) {
        // the Cauchy code of (k, r') holds rows 0..r'-1: take the smallest r'
        // >= rmax with generated kernels, so the decode runs on them
        for (uint32_t r2 = rc; r2 <= emax && k + r2 <= 256; ++r2)
            if (qf::syn_available(k, r2) || qf::bs_available(k, r2)) {
                rc = r2;
                break;
            }
    }
    p->rc = p->cauchy ? rc : emax;
}

// decoder.rs:763-780: the generation in source order -- received systematic
// rows as they came, recovered rows (ridx[m] <- rec row m) at L bytes.
static void decoder_assemble(qf_decoder* d, uint32_t L, uint32_t nrec, const uint16_t* ridx, const uint8_t* rec,
                             uint64_t rec_stride) {
    const uint32_t k = d->k;
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
        memcpy(&d->out[(size_t)i * d->stride], rec + (size_t)m * rec_stride, L);
        d->out_len[i] = L;
    }
    d->decoded = true;
}

// decoder.rs:704-783 for the k accepted rows, on the device.
// Rows [uploaded, accepted) of the pinned host rows to the device, one copy
// (rows is pinned and a slot is not rewritten while its decoder lives).
static int decoder_upload(qf_decoder* d) {
    if (d->uploaded >= d->accepted) return QF_OK;
    const size_t o = (size_t)d->uploaded * d->stride, n = (size_t)(d->accepted - d->uploaded) * d->stride;
    QF_CHECK_HIP(hipMemcpyAsync(d->d_rows + o, d->rows + o, n, hipMemcpyHostToDevice,
                                (hipStream_t)qf_ctx_stream(d->ctx)));
    d->uploaded = d->accepted;
    return QF_OK;
}

// decoder.rs:794-975 for k > 256: the k accepted rows are k - e systematic
// rows and e repair rows; Wiedemann on the e x e block of the erased sources
// (qf_wiedemann.hip), then the recovered rows down.
static int decoder_try_decode_wiedemann(qf_decoder* d) {
    const uint32_t k = d->k;
    hipStream_t st = (hipStream_t)qf_ctx_stream(d->ctx);
    uint32_t L = 0;
    for (uint32_t q = 0; q < k; ++q) L = d->lens[q] > L ? d->lens[q] : L;
    std::vector<uint16_t> E;
    for (uint32_t i = 0; i < k; ++i)
        if (d->sys_slot[i] < 0) E.push_back((uint16_t)i);
    const uint32_t e = (uint32_t)E.size();
    if (e == 0) {   // every source arrived
        decoder_assemble(d, L == 0 ? 1 : L, 0, nullptr, nullptr, 0);
        return QF_OK;
    }
    std::vector<uint32_t> slot(k);
    std::vector<uint8_t> A((size_t)e * k);
    uint32_t p = 0;
    for (uint32_t q = 0; q < k; ++q) {
        if (d->index[q] == k) {
            memcpy(&A[(size_t)p * k], &d->coeffs[(size_t)q * k], k);
            slot[q] = 0x80000000u | p++;
        } else {
            slot[q] = d->index[q];
        }
    }
    if (p != e) return QF_EINVAL;   // k accepted rows: #repairs == #erased
    if (int u = decoder_upload(d)) return u;
    if (d->wrec_rows < e) {
        hipFree(d->d_wrec);
        d->d_wrec = nullptr;
        d->wrec_rows = 0;
        QF_CHECK_HIP(hipMalloc(&d->d_wrec, (size_t)e * d->stride));
        d->wrec_rows = e;
    }
    const int s = qf::wiedemann_decode(d->ctx, k, e, A.data(), E.data(), slot.data(), d->d_rows, d->stride, L,
                                   d->d_wrec, &d->w_tries);
    if (s != QF_OK) return s;   // QF_ERANK: singular, stays undecoded (decoder.rs:852-854)
    std::vector<uint8_t> rec((size_t)e * d->stride);
    QF_CHECK_HIP(hipMemcpyAsync(rec.data(), d->d_wrec, rec.size(), hipMemcpyDeviceToHost, st));
    QF_CHECK_HIP(hipStreamSynchronize(st));
    decoder_assemble(d, L == 0 ? 1 : L, e, E.data(), rec.data(), d->stride);
    return QF_OK;
}

static int decoder_try_decode(qf_decoder* d) {
    const uint32_t k = d->k;
    if (k > 256) return decoder_try_decode_wiedemann(d);
    hipStream_t st = (hipStream_t)qf_ctx_stream(d->ctx);
    const uint32_t emax = k < 128 ? k : 128;
    DecPlan plan;
    decoder_plan(d, &plan);
    const uint32_t L = plan.L;
    if (!plan.cauchy)
        QF_CHECK_HIP(hipMemcpyAsync(d->d_coeffs, d->coeffs.data(), (size_t)k * k, hipMemcpyHostToDevice, st));
    // the rows not on the device yet and the row indices after them, in one
    // copy from pinned memory (slots are contiguous, the indices follow them)
    memcpy(d->h_index, plan.idx.data(), (size_t)k * 2);
    {
        const size_t o = (size_t)d->uploaded * d->stride, end = (size_t)k * d->stride + (size_t)k * 2;
        QF_CHECK_HIP(hipMemcpyAsync(d->d_rows + o, d->rows + o, end - o, hipMemcpyHostToDevice, st));
        d->uploaded = d->accepted;
    }
    qf_decode_shape sh{};
    sh.k = k;
    sh.r = plan.rc;
    sh.L = L;
    sh.max_rows = k;
    sh.row_stride = d->stride;
    sh.rows_gen_stride = (uint64_t)k * d->stride;
    sh.rec_row_stride = d->stride;
    sh.rec_gen_stride = (uint64_t)emax * d->stride;
    int s = qf_decode_batch(d->ctx, &sh, 1, d->d_rows, d->d_index, nullptr, plan.cauchy ? nullptr : d->d_coeffs,
                            d->d_rec, d->d_rec_index, d->d_nrec, d->d_status);
    if (s != QF_OK) return s;
    // status, count, indices and up to rc recovered rows (nrec <= rc): one
    // download into pinned memory, one wait
    const uint32_t nmax = std::min(plan.rc, emax);
    QF_CHECK_HIP(hipMemcpyAsync(d->h_out, d->d_out, kOutMeta + (size_t)nmax * d->stride, hipMemcpyDeviceToHost, st));
    QF_CHECK_HIP(hipStreamSynchronize(st));
    const int32_t status = *reinterpret_cast<const int32_t*>(d->h_out);
    const uint32_t nrec = *reinterpret_cast<const uint32_t*>(d->h_out + 4);
    if (status != QF_OK) return status;  // singular: stays undecoded (decoder.rs:756-758)
    if (nrec > nmax) return qf::device_fail(__FILE__, __LINE__, hipErrorIllegalState);  // internal inconsistency
    decoder_assemble(d, L, nrec, reinterpret_cast<const uint16_t*>(d->h_out + 16), d->h_rec, d->stride);
    return QF_OK;
}

// decoder.rs:679-699 on the host: *slot = the accepted row's slot (its bytes
// are in d->rows), or -1 when the packet is not taken.  Returns what
// add_packet returns when nothing more happens (1 decoded / 0), or an error.
static int decoder_accept(qf_decoder* d, uint64_t id, int is_systematic, const uint8_t* data, uint32_t len,
                          const uint8_t* coeffs, uint32_t coeff_len, int32_t* slot) {
    *slot = -1;
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
    d->lens[q] = len;
    d->accepted++;
    *slot = (int32_t)q;
    return 0;
}

int qf_decoder_add_packet(qf_decoder* d, uint64_t id, int is_systematic, const uint8_t* data,
                          uint32_t len, const uint8_t* coeffs, uint32_t coeff_len) {
    int32_t q = -1;
    const int s = decoder_accept(d, id, is_systematic, data, len, coeffs, coeff_len, &q);
    const bool again = s == 0 && q < 0 && d->retry && !d->decoded && d->accepted == d->k;
    if ((s != 0 || q < 0) && !again) return s;
    // the row stays in the pinned host rows until the generation decodes:
    // one upload of all k rows then, instead of a copy per packet
    if (d->accepted == d->k) {
        d->retry = false;
        int e = decoder_try_decode(d);
        if (e == QF_ERANK) return 0;
        if (e != QF_OK) {
            d->retry = true;
            d->uploaded = 0;
            return e;
        }
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

namespace qf {

namespace {
double wall() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Host copy-out of large send batches: a few persistent workers plus the
// calling thread take items off a shared counter (a single-thread memcpy of
// the ~12 MB of repairs of 1024 windows runs at ~12 GB/s).  QF_COPY_THREADS
// QF_OPT_COPY_THREADS of the context whose batch first uses the pool sets
// the worker count (0: the calling thread alone, -1: auto).
class CopyPool {
  public:
    static CopyPool& get(int64_t threads) {
        static CopyPool p(threads);
        return p;
    }
    // fn(i) for every i < n, across the workers and the calling thread
    void run(uint32_t n, const std::function<void(uint32_t)>& fn) {
        if (th_.empty() || n < 2) {
            for (uint32_t i = 0; i < n; ++i) fn(i);
            return;
        }
        std::lock_guard<std::mutex> one(run_mu_);  // one job at a time (contexts may send concurrently)
        std::unique_lock<std::mutex> lk(mu_);
        job_ = &fn;
        n_ = n;
        next_.store(0);
        busy_ = (uint32_t)th_.size();
        ++gen_;
        lk.unlock();
        cv_.notify_all();
        drain(fn, n);
        lk.lock();
        done_.wait(lk, [&] { return busy_ == 0; });
        job_ = nullptr;
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }

  private:
    explicit CopyPool(int64_t threads) {
        unsigned hw = std::thread::hardware_concurrency();
        unsigned n = threads >= 0 ? (unsigned)threads : std::min(7u, hw > 2 ? hw / 2 - 1 : 0u);
        for (unsigned i = 0; i < n; ++i) th_.emplace_back([this] { loop(); });
    }
    void drain(const std::function<void(uint32_t)>& fn, uint32_t n) {
        for (uint32_t i; (i = next_.fetch_add(1)) < n;) fn(i);
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            const std::function<void(uint32_t)>* fn = job_;
            const uint32_t n = n_;
            lk.unlock();
            drain(*fn, n);
            lk.lock();
            if (--busy_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_, run_mu_;
    std::condition_variable cv_, done_;
    const std::function<void(uint32_t)>* job_ = nullptr;
    std::atomic<uint32_t> next_{0};
    uint32_t n_ = 0, busy_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};
}  // namespace

int encoders_send_batch(qf_ctx* ctx, EncSend* v, uint32_t M) {
    if (!ctx || (M && !v)) return QF_EINVAL;
    if (M == 0) return QF_OK;
    // QF_OPT_SEND_PROFILE of THIS context (per-context sums, printed at qf_ctx_destroy)
    const bool prof = ctx_opt(ctx, QF_OPT_SEND_PROFILE) != 0;
    const double tp0 = prof ? wall() : 0.0;
    for (uint32_t m = 0; m < M; ++m) {
        qf_encoder* e = v[m].e;
        if (!e || e->ctx != ctx || (v[m].len && !v[m].data) || v[m].len > e->max_len) return QF_EINVAL;
        if (e->n > e->k && !window_rows(e, e->n - e->k)) return QF_ERANGE;
    }
    // packets a per-packet add left for the fused send go up before the scatter
    for (uint32_t m = 0; m < M; ++m)
        if (int fs = encoder_flush(v[m].e)) return fs;
    std::unique_lock<std::mutex> lk;
    int s = ctx_lock(ctx, lk);
    if (s) return s;
    hipStream_t st = ctx_stream(ctx);
    // the adds (decoder.rs:164-169) on the host side, and the windows they fill.
    // An encoder that takes several packets in this call (one connection's
    // burst) has its windows overlap: window j of the burst is the k rows
    // ending at its packet j.  Its rows go to a linear staging area instead
    // of the ring -- the newest k-1 rows the ring held before the call, then
    // the burst's packets -- and window j reads rows j' .. j' + k - 1 there
    // unrotated: one launch for the whole burst, as the sliding-window
    // encode.  The ring then keeps only the burst's last k packets.
    struct Win {
        uint32_t m, rot, L;
        uint64_t src_off;   // relative to the staging buffer d; ~0: the encoder's ring
    };
    struct Burst {
        uint32_t B = 0, seen = 0, nold = 0, head0 = 0;
        size_t ext_off = 0;   // relative to d
    };
    std::unordered_map<const qf_encoder*, Burst> bursts;
    for (uint32_t m = 0; m < M; ++m) bursts[v[m].e].B++;
    size_t ext_bytes = 0;
    uint32_t n_old = 0;
    for (auto& kv : bursts) {
        Burst& b = kv.second;
        if (b.B < 2) continue;
        const qf_encoder* e = kv.first;
        b.head0 = e->head;
        b.nold = std::min(e->count, e->k - 1);
        b.ext_off = ext_bytes;   // relative to the staging area for now
        ext_bytes += (size_t)(b.nold + b.B) * e->stride;
        n_old += b.nold;
    }
    std::vector<RingSlot> slots;   // packet copies (second launch)
    std::vector<uint32_t> slot_m;  // their packets
    std::vector<size_t> slot_ext;  // ~0: dst is a ring slot; else the staging row's offset in the burst area
    std::vector<RingSlot> olds;    // ring -> staging copies of the bursts' old rows (first launch)
    slots.reserve(M);
    slot_m.reserve(M);
    slot_ext.reserve(M);
    olds.reserve(n_old);
    std::vector<size_t> pk_src(M);
    std::vector<Win> wins;
    size_t pk = 0;
    const uint64_t kRingSrc = ~0ull;
    for (uint32_t m = 0; m < M; ++m) {
        qf_encoder* e = v[m].e;
        Burst& bu = bursts[e];
        const uint32_t slot = e->head;
        pk_src[m] = pk;   // relative to the packet area for now
        pk += round16(v[m].len);
        e->lens[slot] = v[m].len;
        e->ids[slot] = v[m].id;
        e->head = (e->head + 1) % e->k;
        if (e->count < e->k) e->count++;
        v[m].n_rep = 0;
        const uint32_t j = bu.seen++;
        // the ring copy: every packet of a single add, the last k of a burst
        if (bu.B < 2 || j + e->k >= bu.B) {
            RingSlot rs{};
            rs.dst = e->d_ring + (size_t)slot * e->stride;
            rs.dst2 = e->ring_rot ? nullptr : e->d_ring + (size_t)(slot + e->k) * e->stride;
            rs.len = v[m].len;
            rs.stride = e->stride;
            slots.push_back(rs);
            slot_m.push_back(m);
            slot_ext.push_back(~(size_t)0);
        }
        if (bu.B >= 2) {   // and its row of the burst's staging area
            RingSlot rs{};
            rs.len = v[m].len;
            rs.stride = e->stride;
            slots.push_back(rs);
            slot_m.push_back(m);
            slot_ext.push_back(bu.ext_off + (size_t)(bu.nold + j) * e->stride);
        }
        if (e->count == e->k && e->n > e->k) {
            uint64_t so = kRingSrc;
            uint32_t rot = e->head;
            if (bu.B >= 2) {   // rows nold + j + 1 - k .. nold + j of the burst's staging area
                so = bu.ext_off + (size_t)(bu.nold + j + 1 - e->k) * e->stride;
                rot = 0;
            }
            wins.push_back({m, rot, e->lens[e->head], so});
        }
    }
    // windows grouped by (k, r) class, repairs packed L-rounded per window
    std::sort(wins.begin(), wins.end(), [&](const Win& a, const Win& b) {
        const qf_encoder *x = v[a.m].e, *y = v[b.m].e;
        return x->k != y->k ? x->k < y->k : x->n != y->n ? x->n < y->n : a.m < b.m;
    });
    const uint32_t n_slots = (uint32_t)slots.size(), n_olds = n_old;
    const size_t slots_off = 0, olds_off = round16((uint32_t)(sizeof(RingSlot) * n_slots));
    const size_t wins_off = olds_off + round16((uint32_t)(sizeof(RingSlot) * n_olds));
    const size_t pk_off = wins_off + round16((uint32_t)(sizeof(RingWin) * wins.size()));
    const size_t ext_off0 = (pk_off + pk + 255) & ~(size_t)255;
    const size_t rep_off0 = (ext_off0 + ext_bytes + 255) & ~(size_t)255;
    std::vector<size_t> rep_off(wins.size());
    size_t rep_bytes = 0;
    for (size_t w = 0; w < wins.size(); ++w) {
        rep_off[w] = rep_off0 + rep_bytes;
        rep_bytes += (size_t)(v[wins[w].m].e->n - v[wins[w].m].e->k) * round16(wins[w].L);
    }
    uint8_t *h = nullptr, *d = nullptr;
    const double tpa = prof ? wall() : 0.0;
    if ((s = ctx_desc_buffers(ctx, rep_off0 + rep_bytes, &h, &d)) != QF_OK) return s;
    const double tpb = prof ? wall() : 0.0;
    for (uint32_t m = 0; m < M; ++m) {
        uint8_t* dst = h + pk_off + pk_src[m];
        const uint32_t n = v[m].len, n16 = round16(n);
        if (n) memcpy(dst, v[m].data, n);
        if (n16 > n) memset(dst + n, 0, n16 - n);
    }
    for (uint32_t i = 0; i < n_slots; ++i) {
        slots[i].src_off = pk_off + pk_src[slot_m[i]];
        if (slot_ext[i] != ~(size_t)0) slots[i].dst = d + ext_off0 + slot_ext[i];
    }
    for (auto& kv : bursts) {   // old rows, oldest first: ring slots head0 - nold .. head0 - 1
        const Burst& b = kv.second;
        if (b.B < 2) continue;
        const qf_encoder* e = kv.first;
        for (uint32_t t = 0; t < b.nold; ++t) {
            const uint32_t slot = (b.head0 + e->k - b.nold + t) % e->k;
            RingSlot rs{};
            rs.src_off = (uint64_t)(uintptr_t)(e->d_ring + (size_t)slot * e->stride) - (uint64_t)(uintptr_t)d;   // wraps below d
            rs.dst = d + ext_off0 + b.ext_off + (size_t)t * e->stride;
            rs.len = e->stride;
            rs.stride = e->stride;
            olds.push_back(rs);
        }
    }
    memcpy(h + slots_off, slots.data(), sizeof(RingSlot) * n_slots);
    if (n_olds) memcpy(h + olds_off, olds.data(), sizeof(RingSlot) * n_olds);
    const double tpc = prof ? wall() : 0.0;
    RingWin* hw = reinterpret_cast<RingWin*>(h + wins_off);
    for (size_t w = 0; w < wins.size(); ++w) {
        const qf_encoder* e = v[wins[w].m].e;
        hw[w].src_off = wins[w].src_off == kRingSrc ? (uint64_t)(uintptr_t)e->d_ring - (uint64_t)(uintptr_t)d   // wraps when the ring is below d
                                                    : ext_off0 + wins[w].src_off;
        hw[w].rep_off = rep_off[w];
        hw[w].rot = wins[w].rot;
        hw[w].L = wins[w].L;
        hw[w].src_row_stride = e->stride;
        hw[w].rep_row_stride = round16(wins[w].L);
    }
    if ((s = ctx_desc_upload(ctx, pk_off + pk)) != QF_OK) return s;
    const double tp1 = prof ? wall() : 0.0;
    // the bursts' old rows leave the rings before their packets overwrite them
    if (n_olds) QF_CHECK_HIP(launch_ring_scatter(d, reinterpret_cast<const RingSlot*>(d + olds_off), n_olds, st));
    QF_CHECK_HIP(launch_ring_scatter(d, reinterpret_cast<const RingSlot*>(d + slots_off), n_slots, st));
    for (size_t w0 = 0; w0 < wins.size();) {
        const qf_encoder* e = v[wins[w0].m].e;
        size_t w1 = w0;
        uint32_t max_L = 0;
        while (w1 < wins.size() && v[wins[w1].m].e->k == e->k && v[wins[w1].m].e->n == e->n)
            max_L = std::max(max_L, wins[w1++].L);
        s = encode_ring_windows(ctx, e->k, e->n - e->k, (uint32_t)(w1 - w0), max_L, d, d,
                                reinterpret_cast<const RingWin*>(d + wins_off) + w0);
        if (s != QF_OK) return s;
        w0 = w1;
    }
    const double tp2 = prof ? wall() : 0.0;
    // the repairs out (decoder.rs:172-275): window[0].len bytes, ids after the newest
    auto copy_out = [&](uint32_t w) {
        EncSend& x = v[wins[w].m];
        const qf_encoder* e = x.e;
        const uint32_t r = e->n - e->k, L = wins[w].L, Lr = round16(L);
        const uint64_t newest = x.id;   // the window's newest packet is the one that filled it
        for (uint32_t q = 0; q < r; ++q) {
            if (L) memcpy(x.rep_data + (size_t)q * x.rep_stride, h + rep_off[w] + (size_t)q * Lr, L);
            if (x.rep_coeffs) memcpy(x.rep_coeffs + (size_t)q * x.coeff_stride, e->win.data() + (size_t)q * e->k, e->k);
            qf_packet_desc& dd = x.rep_desc[q];
            dd.id = newest + 1 + q;
            dd.len = L;
            dd.coeff_len = e->k;
            dd.is_systematic = 0;
            dd.reserved = 0;
        }
        x.n_rep = r;
    };
    // download in chunks of windows, each copied out on the host while the
    // next one is in flight; large chunks go through the copy workers
    const uint32_t nw = (uint32_t)wins.size();
    const uint32_t max_chunks = (uint32_t)ctx_opt(ctx, QF_OPT_SEND_CHUNKS);
    const uint32_t chunks = nw == 0 ? 0 : std::max(1u, std::min<uint32_t>(max_chunks, (uint32_t)(rep_bytes >> 20)));
    hipEvent_t* ev = nullptr;
    if (chunks && (s = ctx_send_events(ctx, chunks, &ev)) != QF_OK) return s;
    std::vector<uint32_t> cw(chunks + 1, nw);  // first window of each chunk
    cw[0] = 0;
    for (uint32_t c = 1, w = 0; c < chunks; ++c) {
        const size_t target = rep_bytes * c / chunks;
        while (w < nw && rep_off[w] - rep_off0 < target) ++w;
        cw[c] = w;
    }
    for (uint32_t c = 0; c < chunks; ++c) {
        const size_t b0 = cw[c] < nw ? rep_off[cw[c]] : rep_off0 + rep_bytes;
        const size_t b1 = cw[c + 1] < nw ? rep_off[cw[c + 1]] : rep_off0 + rep_bytes;
        if (b1 > b0) QF_CHECK_HIP(hipMemcpyAsync(h + b0, d + b0, b1 - b0, hipMemcpyDeviceToHost, st));
        QF_CHECK_HIP(hipEventRecord(ev[c], st));
    }
    double t_wait = 0.0;
    for (uint32_t c = 0; c < chunks; ++c) {
        const double tw = prof ? wall() : 0.0;
        QF_CHECK_HIP(hipEventSynchronize(ev[c]));
        if (prof) t_wait += wall() - tw;
        const uint32_t w0 = cw[c], n = cw[c + 1] - cw[c];
        if ((size_t)(chunks > 1 ? rep_bytes / chunks : rep_bytes) >= ((size_t)1 << 20)) {
            CopyPool::get(ctx_opt(ctx, QF_OPT_COPY_THREADS)).run(n, [&](uint32_t i) { copy_out(w0 + i); });
        } else {
            for (uint32_t i = 0; i < n; ++i) copy_out(w0 + i);
        }
    }
    const double tp3 = tp2 + t_wait;
    SendProfile* sp = ctx_send_profile(ctx);
    if (prof && rep_bytes && ++sp->seen > 4) {   // steady state: windows full, buffers grown
        const double tp4 = wall();
        sp->calls++;
        sp->t[0] += tp1 - tp0;
        sp->u[0] += tpa - tp0;
        sp->u[1] += tpb - tpa;
        sp->u[2] += tpc - tpb;
        sp->u[3] += tp1 - tpc;
        sp->t[1] += tp2 - tp1;
        sp->t[2] += tp3 - tp2;
        sp->t[3] += tp4 - tp3;
    }
    return QF_OK;
}

int decoders_add_batch(qf_ctx* ctx, DecAdd* v, uint32_t M) {
    if (!ctx || (M && !v)) return QF_EINVAL;
    if (M == 0) return QF_OK;
    {
        std::vector<const qf_decoder*> ds(M);
        for (uint32_t m = 0; m < M; ++m) {
            if (!v[m].d || v[m].d->ctx != ctx) return QF_EINVAL;
            ds[m] = v[m].d;
        }
        std::sort(ds.begin(), ds.end());
        if (std::adjacent_find(ds.begin(), ds.end()) != ds.end()) return QF_EINVAL;   // one packet per decoder
    }
    {
        std::unique_lock<std::mutex> lk;
        int s = ctx_lock(ctx, lk);   // device current
        if (s) return s;
    }
    // decoder.rs:679-699 on the host, in order
    struct Up {
        uint32_t m, slot;
    };
    std::vector<Up> up;
    std::vector<uint32_t> done;          // packets whose decoder now holds k rows
    // a failure before the decodes: the rows of this call's packets are on
    // the host only, so every decoder touched re-uploads all its rows on its
    // next add, and one that holds k rows decodes then
    auto abandon = [&](int err) {
        for (const Up& u : up) {
            qf_decoder* d = v[u.m].d;
            d->uploaded = 0;
            if (d->accepted == d->k && !d->decoded) d->retry = true;
        }
        for (uint32_t m : done) {
            v[m].d->uploaded = 0;
            v[m].d->retry = true;
            v[m].result = err;
        }
    };
    size_t pk = 0;
    for (uint32_t m = 0; m < M; ++m) {
        DecAdd& x = v[m];
        int32_t q = -1;
        const uint32_t before = x.d->uploaded;
        x.result = decoder_accept(x.d, x.id, x.is_systematic, x.data, x.len, x.coeffs, x.coeff_len, &q);
        if (q < 0) {
            // a decoder whose last decode failed on the device: its rows go up
            // again (pinned host copy) and it decodes with this batch
            qf_decoder* d = x.d;
            if (x.result == 0 && d->retry && !d->decoded && d->accepted == d->k) {
                d->retry = false;
                if (int us = decoder_upload(d)) {
                    d->retry = true;
                    x.result = us;
                    continue;
                }
                done.push_back(m);
            }
            continue;
        }
        // rows a per-packet add left on the host go up first (stream order)
        if (before < (uint32_t)q) {
            const uint32_t acc = x.d->accepted;
            x.d->accepted = (uint32_t)q;
            const int us = decoder_upload(x.d);
            x.d->accepted = acc;
            if (us) {
                x.d->uploaded = 0;
                if (x.d->accepted == x.d->k) x.d->retry = true;
                abandon(us);
                return us;
            }
        }
        x.d->uploaded = (uint32_t)q + 1;   // the scatter below writes slot q
        up.push_back({m, (uint32_t)q});
        pk += round16(x.len);
        if (x.d->accepted == x.d->k) done.push_back(m);
    }
    // decode plans: Cauchy generations go into one heterogeneous decode
    std::vector<DecPlan> plans(done.size());
    std::vector<uint32_t> cau, expl;
    size_t ri_n = 0, ri_pad = 0, rec_rows = 0, rec_idx = 0;
    for (size_t t = 0; t < done.size(); ++t) {
        decoder_plan(v[done[t]].d, &plans[t]);
        // (k > 256: the Wiedemann strategy, per generation, whatever the rows)
        if (plans[t].cauchy && v[done[t]].d->k <= 256) {
            cau.push_back((uint32_t)t);
            const qf_decoder* d = v[done[t]].d;
            ri_n += d->k;
            rec_idx += std::min(d->k, plans[t].rc);
            rec_rows += (size_t)std::min(d->k, plans[t].rc) * d->stride;
        } else {
            expl.push_back((uint32_t)t);
        }
    }
    (void)ri_pad;
    const size_t n_up = up.size(), G = cau.size();
    const size_t o_slots = 0, o_ri = round16((uint32_t)(sizeof(RingSlot) * n_up));
    const size_t o_pk = o_ri + ((ri_n * 2 + 255) & ~(size_t)255);
    const size_t o_out = (o_pk + pk + 255) & ~(size_t)255;            // downloads from here
    const size_t o_nrec = o_out, o_st = o_nrec + 4 * G, o_ci = (o_st + 4 * G + 255) & ~(size_t)255;
    const size_t o_rec = (o_ci + 2 * rec_idx + 255) & ~(size_t)255;
    const size_t total = o_rec + rec_rows;
    uint8_t *h = nullptr, *dv = nullptr;
    int s = ctx_recv_buffers(ctx, total, &h, &dv);
    if (s != QF_OK) {
        abandon(s);
        return s;
    }
    hipStream_t st = ctx_stream(ctx);
    RingSlot* hs = reinterpret_cast<RingSlot*>(h + o_slots);
    size_t off = 0;
    for (size_t u = 0; u < n_up; ++u) {
        const DecAdd& x = v[up[u].m];
        qf_decoder* d = x.d;
        const uint32_t n16 = round16(x.len);
        if (x.len) memcpy(h + o_pk + off, x.data, x.len);
        if (n16 > x.len) memset(h + o_pk + off + x.len, 0, n16 - x.len);
        hs[u].src_off = o_pk + off;
        hs[u].dst = d->d_rows + (size_t)up[u].slot * d->stride;
        hs[u].dst2 = nullptr;
        hs[u].len = x.len;
        hs[u].stride = d->stride;
        off += n16;
    }
    // row indices of the Cauchy decodes, and their descriptors
    std::vector<qf_dec_desc> descs(G);
    const uint8_t* rows_base = nullptr;
    for (size_t c = 0; c < G; ++c) {
        const qf_decoder* d = v[done[cau[c]]].d;
        if (!rows_base || d->d_rows < rows_base) rows_base = d->d_rows;
    }
    uint16_t* hri = reinterpret_cast<uint16_t*>(h + o_ri);
    size_t ri_o = 0, ci_o = 0, rr_o = 0;
    for (size_t c = 0; c < G; ++c) {
        const DecPlan& pl = plans[cau[c]];
        const qf_decoder* d = v[done[cau[c]]].d;
        memcpy(hri + ri_o, pl.idx.data(), (size_t)d->k * 2);
        qf_dec_desc& q = descs[c];
        q.k = d->k;
        q.r = pl.rc;
        q.L = pl.L;
        q.n_rows = d->k;
        q.rows_offset = (uint64_t)(d->d_rows - rows_base);
        q.row_stride = d->stride;
        q.row_index_offset = ri_o;
        q.rec_offset = rr_o;
        q.rec_row_stride = d->stride;
        q.rec_index_offset = ci_o;
        ri_o += d->k;
        ci_o += std::min(d->k, pl.rc);
        rr_o += (size_t)std::min(d->k, pl.rc) * d->stride;
    }
    {
        hipError_t e = o_pk + pk ? hipMemcpyAsync(dv, h, o_pk + pk, hipMemcpyHostToDevice, st) : hipSuccess;
        if (e == hipSuccess) e = launch_ring_scatter(dv, reinterpret_cast<const RingSlot*>(dv + o_slots), (uint32_t)n_up, st);
        if (e != hipSuccess) {
            const int err = qf::device_fail(__FILE__, __LINE__, e);
            abandon(err);
            ctx_recv_release(ctx);
            return err;
        }
    }
    // a failed batch decode: every connection whose generation was in it gets
    // the error as its status, and its decoder retries on its next packet
    // (rows re-uploaded from the pinned host copy); the call goes on with
    // the explicit-coefficient generations
    auto fail_cauchy = [&](int err) {
        for (size_t c = 0; c < G; ++c) {
            DecAdd& x = v[done[cau[c]]];
            x.result = err;
            x.d->retry = true;
            x.d->uploaded = 0;
        }
    };
    bool failed = false;
    if (G) {
        s = qf_decode_batch_desc(ctx, descs.data(), (uint32_t)G, rows_base, reinterpret_cast<const uint16_t*>(dv + o_ri),
                                 dv + o_rec, reinterpret_cast<uint16_t*>(dv + o_ci),
                                 reinterpret_cast<uint32_t*>(dv + o_nrec), reinterpret_cast<int32_t*>(dv + o_st));
        if (s == QF_OK) {
            hipError_t e = hipMemcpyAsync(h + o_out, dv + o_out, total - o_out, hipMemcpyDeviceToHost, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            if (e != hipSuccess) s = qf::device_fail(__FILE__, __LINE__, e);
        }
        if (s != QF_OK) {
            fail_cauchy(s);
            failed = true;
        }
    }
    if (G && !failed) {
        const uint32_t* nrec = reinterpret_cast<const uint32_t*>(h + o_nrec);
        const int32_t* stt = reinterpret_cast<const int32_t*>(h + o_st);
        for (size_t c = 0; c < G; ++c) {
            DecAdd& x = v[done[cau[c]]];
            const qf_dec_desc& q = descs[c];
            if (stt[c] == QF_OK) {
                decoder_assemble(x.d, q.L, nrec[c], reinterpret_cast<const uint16_t*>(h + o_ci) + q.rec_index_offset,
                                 h + o_rec + q.rec_offset, q.rec_row_stride);
                x.result = 1;
            } else {
                x.result = stt[c] == QF_ERANK ? 0 : stt[c];   // singular: stays undecoded (decoder.rs:756-758)
            }
        }
    }
    if ((s = ctx_recv_release(ctx)) != QF_OK) return s;
    // explicit coefficient rows: the per-generation path (rows are on the device, stream order)
    for (uint32_t t : expl) {
        DecAdd& x = v[done[t]];
        const int e = decoder_try_decode(x.d);
        if (e != QF_OK && e != QF_ERANK) {
            x.d->retry = true;
            x.d->uploaded = 0;
        }
        x.result = e == QF_ERANK ? 0 : (e != QF_OK ? e : (x.d->decoded ? 1 : 0));
    }
    return QF_OK;
}

}  // namespace qf
