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
int encode_ring_window(qf_ctx* ctx, uint32_t k, uint32_t first, uint32_t count, uint32_t L,
                       const uint8_t* ring, uint64_t stride, uint32_t rot, uint8_t* rep, uint64_t rep_stride);
// Whether the small-batch encode is enabled (QF_ENCODE_SMALL != 0).
bool small_encode_enabled();

}  // namespace qf
