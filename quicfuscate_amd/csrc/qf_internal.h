// qf_internal.h -- context services for the library's other translation
// units (defined in qf_api.hip; not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>
#include <string>

#include "qf_fec.h"

namespace qf {

// Locks the context and makes its device current.
int ctx_lock(qf_ctx* ctx, std::unique_lock<std::mutex>& lk);
hipStream_t ctx_stream(qf_ctx* ctx);
int ctx_num_cus(qf_ctx* ctx);
// The context's device workspace, grown to at least `bytes` (shared with the
// decode paths; valid until the next call on this context).
int ctx_work(qf_ctx* ctx, size_t bytes, uint8_t** out);
// GF(2^16) tables on the device, built on first use: log[65536] (log[0] =
// 0xFFFF, no product) and exp[2 * 65535] (exp[i + 65535] = exp[i]).
int ctx_gf16_tables(qf_ctx* ctx, const uint16_t** log, const uint16_t** exp);
// The context's 256 split-table records (8 dwords each, gf256_tables.h).
const uint32_t* ctx_tab256(qf_ctx* ctx);
// A device buffer of >= bytes for GF(2^16) input rows in log form (its own
// allocation, so it can sit beside the workspace; valid until the next call).
int ctx_gf16_logrows(qf_ctx* ctx, size_t bytes, uint8_t** out);
// The context's value of option `opt` (QF_OPT_*, qf_ctx_set_option).
int64_t ctx_opt(qf_ctx* ctx, int opt);
// qf_ctx_profile bracketing of a launch.
hipEvent_t ctx_prof_begin(qf_ctx* ctx, hipStream_t st);
void ctx_prof_end(qf_ctx* ctx, hipStream_t st, hipEvent_t ev, const std::string& name);

}  // namespace qf

namespace qf {

// qf_encode16_batch over a ring of k source slots: window position i in slot
// (rot + i) % k, repairs = Cauchy rows first..first+r-1 (coeff_rxk must be
// NULL for first/rot != 0); coeff_be_dev (optional, device) receives each
// repair's big-endian coefficient block in window order.  (qf_gf16.hip)
int encode16_window(qf_ctx* ctx, const qf_encode_shape* sh, uint32_t G, const uint8_t* src, uint8_t* rep,
                    const uint16_t* coeff_rxk, uint32_t first, uint32_t rot, uint8_t* coeff_be_dev);

// One GF(2^8) window over a ring of k source slots (slot stride `stride`):
// window position i in slot (rot + i) % k; repairs = Cauchy rows
// first..first+count-1 into rep (row stride rep_stride), on the small-batch
// kernel.  QF_ERANGE when k + first + count > 256.  (qf_api.hip)
// fresh (fused per-packet send): window position k - 1 is the host packet
// fresh (fresh_units zero-padded 16-byte units, <= SEND_PKT_UNITS), passed in
// the kernel arguments and written into the ring slot fresh_dst; rep is then
// a host-coherent buffer of whole 16-byte units per row.
int encode_ring_window(qf_ctx* ctx, uint32_t k, uint32_t first, uint32_t count, uint32_t L,
                       const uint8_t* ring, uint64_t stride, uint32_t rot, uint8_t* rep, uint64_t rep_stride,
                       const uint8_t* fresh = nullptr, uint8_t* fresh_dst = nullptr, uint32_t fresh_units = 0);
// Whether the small-batch encode is enabled (QF_OPT_ENCODE_SMALL != 0).
bool small_encode_enabled(qf_ctx* ctx);

// Multi-connection send batches (qf_objects.hip).  The caller holds the
// context lock (ctx_lock) across these.
// The context's per-call metadata buffers, pinned host and device, `bytes`
// each, once the previous call's upload has landed.
int ctx_desc_buffers(qf_ctx* ctx, size_t bytes, uint8_t** h, uint8_t** d);
// The first `bytes` of the host buffer to the device buffer, on the context stream.
int ctx_desc_upload(qf_ctx* ctx, size_t bytes);
// Receive batches: pinned + device buffers of >= bytes each, once the
// previous user's host reads/writes are done (ctx_recv_release records that
// point on the context stream).  The caller does not hold the context lock.
int ctx_recv_buffers(qf_ctx* ctx, size_t bytes, uint8_t** h, uint8_t** d);
int ctx_recv_release(qf_ctx* ctx);
// At least n events of the context (download chunks of a send batch).
int ctx_send_events(qf_ctx* ctx, uint32_t n, hipEvent_t** out);
// Small-batch encode of G ring windows of one (k, r) class, repairs = Cauchy
// rows 0..r-1: window g per wins[g] (device records), rings addressed from
// src, repairs from rep; max_L (>= every window's L) sizes the grid.
int encode_ring_windows(qf_ctx* ctx, uint32_t k, uint32_t r, uint32_t G, uint32_t max_L, const uint8_t* src,
                        uint8_t* rep, const struct RingWin* wins);

// One connection's share of a send batch: a source packet for encoder e, and
// where repairs 0..n-k-1 of its window go when the add fills it.
struct EncSend {
    qf_encoder* e;
    uint64_t id;
    const uint8_t* data;
    uint32_t len;
    uint8_t* rep_data;            // rows rep_stride apart, >= window[0].len bytes each
    uint32_t rep_stride;
    uint8_t* rep_coeffs;          // nullable: k coefficient bytes per repair, coeff_stride apart
    uint32_t coeff_stride;
    qf_packet_desc* rep_desc;
    uint32_t n_rep;               // out: repairs emitted (0, or n - k)
};
// qf_encoder_add_source_packet + qf_encoder_generate_repairs(0, n - k) for M
// distinct encoders of ctx (lengths already checked): one upload, one ring
// scatter, one small-batch encode per (k, r) class, one download.  The
// caller does not hold the context lock.
int encoders_send_batch(qf_ctx* ctx, EncSend* v, uint32_t M);

// One packet for each of M distinct GF(2^8) decoders of ctx
// (qf_decoder_add_packet semantics, result per packet: 1 decoded, 0 not, < 0
// error): the accepted rows go up in one copy and one scatter; decoders that
// reach k rows decode together (one qf_decode_batch_desc over the Cauchy
// ones), with one download of all their outputs.
struct DecAdd {
    qf_decoder* d;
    uint64_t id;
    int is_systematic;
    const uint8_t* data;
    uint32_t len;
    const uint8_t* coeffs;
    uint32_t coeff_len;
    int result;
};
int decoders_add_batch(qf_ctx* ctx, DecAdd* v, uint32_t M);

// The k > 256 strategy of the GF(2^8) decoder (qf_wiedemann.hip,
// decoder.rs:794-975): k accepted rows on the device (slot q at q * stride,
// zero padded), e of them repairs with coefficient rows A_ek (e x k, host, in
// repair order), E the e erased sources ascending (host), slot[q] = source
// index of a systematic slot or 0x80000000 | repair ordinal (host).  Writes
// recovered row t (source E[t]) to d_rec + t * stride (L bytes, zero padded
// to 16).  QF_ERANK when the system is singular.  Takes the context lock;
// asynchronous on the context stream once it returns QF_OK.
int wiedemann_decode(qf_ctx* ctx, uint32_t k, uint32_t e, const uint8_t* A_ek, const uint16_t* E,
                     const uint32_t* slot, const uint8_t* d_rows, uint64_t stride, uint32_t L, uint8_t* d_rec,
                     uint32_t* tries_out);

}  // namespace qf
