// qf_bs.h -- bit-sliced Cauchy encode kernels (generated gfx950 assembly).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "qf_fec.h"
#include "qf_kernels.h"

namespace qf {

struct BsCache {
    static const int kMax = 128;   // >= the entries of qf_bs_table (build_lib.py checks)
    hipModule_t mod[kMax] = {};
    hipFunction_t fn[kMax] = {};
    // the owning context's options (QF_OPT_*, qf_ctx_set_option)
    const int64_t* opt = nullptr;
    int64_t get(int o) const { return opt ? opt[o] : 0; }
};

// Is there a specialised kernel for the Cauchy matrix of (k, r)?
bool bs_available(uint32_t k, uint32_t r);
// Kernel symbol of that configuration (nullptr if none).
const char* bs_name(uint32_t k, uint32_t r, bool fft = false);
// Lane units per row of the padded lane space: ceil(L/16) rounded up to 8 (128 B).
uint32_t bs_padded_units(uint32_t L);
// Does every repair row's zero tail stay inside its own row / generation?
bool bs_zero_tail_fits(uint32_t r, uint32_t L, uint64_t drs, uint64_t dgs);
// Encode G generations (rows of L >= 32 bytes; strides and generation strides
// < 2^32, 16-byte aligned; G * L / 16 < 2^31), one launch per pass of at most
// 16 repairs.  zero_tail: also write zeros to bytes [L, 16 * bs_padded_units(L))
// of every repair row (needs drs >= that); required when L % 16 != 0 (the
// last unit of each source row is then read whole, up to round_up(L, 16)).
hipError_t bs_launch(BsCache& cache, int num_cus, hipStream_t st, uint32_t k, uint32_t r,
                     const uint8_t* src, uint8_t* dst, uint64_t sgs, uint64_t dgs, uint64_t srs,
                     uint64_t drs, uint32_t L, uint32_t G, bool zero_tail, const uint64_t* src_offs = nullptr,
                     const uint64_t* dst_offs = nullptr, const char** name_out = nullptr);
// (src_offs / dst_offs: generation offset tables -- generation g at src +
// src_offs[g] / dst + dst_offs[g] instead of g * gen_stride -- or nullptr)
// Decode stage A: syndromes of the accepted repairs (bs_codegen.py "syn").
// zero: >= L zero bytes (read in place of rows a generation does not have).
// srs >= 16 * bs_padded_units(L): syndromes are computed over the padded lane
// space (the tail bytes are junk).
bool syn_available(uint32_t k, uint32_t r);
// Syndromes for long rows (padded units >= 128) with the slot map read by
// the scalar unit, every repair pass of (k, r); items whose generations'
// bound (1 + largest accepted repair) <= a pass's first repair skip it.
bool synw_available(uint32_t k, uint32_t r);
hipError_t synw_launch(BsCache& cache, int num_cus, hipStream_t st, uint32_t k, uint32_t r,
                       const uint8_t* rows, uint8_t* syn, uint64_t rgs, uint64_t sgs, uint64_t rs,
                       uint64_t srs, uint32_t L, uint32_t G, const uint8_t* smap, uint32_t map_stride,
                       const uint8_t* zero, const uint32_t* bound, const uint64_t* rows_offs);
const char* syn_name(uint32_t k, uint32_t r);
uint32_t syn_map_stride(uint32_t k, uint32_t r);
hipError_t syn_launch(BsCache& cache, int num_cus, hipStream_t st, uint32_t k, uint32_t r,
                      const uint8_t* rows, uint8_t* syn, uint64_t rgs, uint64_t sgs, uint64_t rs,
                      uint64_t srs, uint32_t L, uint32_t G, const uint8_t* smap, uint32_t map_stride,
                      const uint8_t* zero, const uint64_t* rows_offs = nullptr);
// Fused decode (bs_codegen.py "dec"): syndromes of the accepted repairs,
// then C[J, E] x = s solved in registers by the per-generation LU records of
// k_decode_prepare_cauchy (lu_out), recovered rows stored to
// rec + g * rec_gs + rank * rec_rs.  Only the payload bytes [0, L) of a
// recovered row are written.  L % 16 != 0 (lane-chunk kernels only): rows are
// read in whole 16-byte units, so they must start 16-byte aligned.
bool dec_available(uint32_t k, uint32_t r);
// the kernel dec_launch runs for (k, r, L) and, given G and num_cus, that batch size
const char* dec_name(const BsCache* cache, uint32_t k, uint32_t r, uint32_t L = 0, uint32_t G = 0,
                     int num_cus = 0);
hipError_t dec_launch(BsCache& cache, int num_cus, hipStream_t st, uint32_t k, uint32_t r,
                      const uint8_t* rows, uint8_t* rec, uint64_t rgs, uint64_t rec_gs, uint64_t rs,
                      uint64_t rec_rs, uint32_t L, uint32_t G, const uint8_t* smap, uint32_t map_stride,
                      const uint8_t* zero, const uint8_t* lu, uint32_t lu_stride, const uint32_t* tab256,
                      const uint64_t* rows_offs = nullptr, const uint64_t* rec_offs = nullptr);
// Decode payload pass x_E = D s (the k_combine_slots records of one pass)
// bit-sliced with wave-uniform coefficients (bs_codegen.py "cmb"): one
// generation per item, units q and q + Q of a row per lane.  idxtab: the
// 256 x 64-byte plane-index table (bs_codegen.cmb_index_table).  Rows are
// read in whole 16-byte units (the unit holding byte L - 1 too); only bytes
// [0, L) of the output rows are written.
// passes > 1: every pass in one pass-major launch (qf_combine_bs_r16_pm):
// pass p takes the records at a.coef + p * pass_stride and writes output rows
// 16 p .. of each generation (a.pass must be 0).
bool cmb_available();
bool cmb_pass_major_available();
// The pass-major launch covers at most kCmbMaxPasses passes (the generated
// loop), and advances dst by 16 rows per pass in a 32-bit SGPR: callers fall
// back to one launch per pass when this is false.
constexpr uint32_t kCmbMaxPasses = 4;
bool cmb_pass_major_ok(uint32_t passes, uint64_t dst_row_stride, uint64_t pass_stride);
// e_max: the largest n_out of the batch; 16 < e_max <= 24 over two passes
// runs the wide single pass (QF_COMBINE_WIDE) when the library holds it and
// cmb_wide_ok says so
bool cmb_wide_ok(BsCache& cache, const CombineSlotsArgs& a, uint32_t passes, uint64_t pass_stride, uint32_t e_max);
// the kernel cmb_launch would run for these arguments (profiling labels)
const char* cmb_kernel_name(BsCache& cache, const CombineSlotsArgs& a, uint32_t passes = 1, uint64_t pass_stride = 0,
                            uint32_t e_max = 0);
hipError_t cmb_launch(BsCache& cache, int num_cus, hipStream_t st, const CombineSlotsArgs& a,
                      const uint32_t* idxtab, uint32_t passes = 1, uint64_t pass_stride = 0,
                      uint32_t e_max = 0);
void bs_unload(BsCache& cache);

}  // namespace qf
