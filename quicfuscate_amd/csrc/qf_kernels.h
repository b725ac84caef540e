// qf_kernels.h -- kernel argument blocks and launch wrappers (internal).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qf {

// Encode / uniform combination:
//   dst[g][j] = XOR_i C[j][i] * src[g][i]   for j < r_active, i < k
// tabs: k_pad * R records of 8 dwords, record (i, j) at (i*R + j)*8, zero
// records for i >= k.  Lanes map over units f = g*Lu + u (16 bytes each).
struct CombineUniformArgs {
    const uint8_t* src;
    uint64_t src_gen_stride;
    uint64_t src_row_stride;
    uint8_t* dst;
    uint64_t dst_gen_stride;
    uint64_t dst_row_stride;
    const uint32_t* tabs;
    uint32_t k;
    uint32_t k_pad;
    uint32_t r_active;
    uint32_t L;
    uint32_t Lu;
    uint32_t pad0;
    uint64_t total_units;
    // generation offset tables (nullptr: g * gen_stride), the heterogeneous
    // batch API: generation g starts at src + src_offs[g] / dst + dst_offs[g]
    const uint64_t* src_offs = nullptr;
    const uint64_t* dst_offs = nullptr;
};

// Decode payload pass (one 16-output pass):
//   dst[g][j] = XOR_s coef[g][s][j] * rows[g][s]   for j < n_out[g]-16*pass
// coef: 16 coefficient bytes per slot, slot s of generation g at
// coef + g*coef_gen_stride + s*16.  Slots >= bound[g] are not read.
struct CombineSlotsArgs {
    const uint8_t* rows;
    uint64_t rows_gen_stride;
    uint64_t row_stride;
    uint8_t* dst;
    uint64_t dst_gen_stride;
    uint64_t dst_row_stride;
    const uint8_t* coef;
    uint64_t coef_gen_stride;
    const uint32_t* n_out;
    const uint32_t* bound;
    const uint32_t* tab256;
    uint32_t pass;
    uint32_t L;
    uint32_t Lu;
    uint32_t zero_slot;  // index of an all-zero coefficient record
    uint64_t total_units;
    const uint64_t* rows_offs = nullptr;  // generation offset tables (nullptr: strided)
    const uint64_t* dst_offs = nullptr;
};

struct PrepareArgs {
    const uint16_t* row_index;
    const uint32_t* n_rows;
    const uint8_t* row_coeffs;
    const uint8_t* explog;  // exp[512] then log[256]
    uint8_t* coef_out;      // [pass][G][coef_gen_stride]
    uint64_t coef_gen_stride;
    uint32_t* n_out;
    uint32_t* bound;
    uint16_t* rec_index;    // [G][e_max]
    int32_t* status;
    uint32_t k;
    uint32_t e_max;   // output capacity min(k, r)
    uint32_t rep_limit;  // repair index j = row_index - k must be < rep_limit
    uint32_t e_lds;   // matrix rows held in LDS, min(k, 128)
    uint32_t max_rows;
    uint32_t max_rows_pad;
    uint32_t passes;
    uint32_t G;
};

// Decode control for the reference's Cauchy code (no row_coeffs): row
// acceptance as k_decode_prepare, then the closed-form inverse of the square
// Cauchy submatrix C[J, E] (no elimination).  Outputs the slot map of the
// syndrome kernel and the stage-B coefficient records (slot j = syndrome of
// repair j, record r all zero).
struct PrepareCauchyArgs {
    const uint16_t* row_index;
    const uint32_t* n_rows;
    const uint8_t* explog;
    uint8_t* coef_out;      // [pass][G][(r + 1) * 16], passes of 16 outputs (e_max <= 64)
    uint8_t* smap;          // [G][map_stride]: k source slots, r repair slots, 0xFF absent
    uint32_t* n_out;
    uint32_t* bound;
    uint16_t* rec_index;    // [G][e_max]
    int32_t* status;
    uint32_t k, r;
    uint32_t e_max;
    uint32_t max_rows;      // <= 255
    uint32_t map_stride;
    uint32_t G;
    // fused decode (qf_cauchy_dec_*): when lu_out != nullptr the kernel
    // writes the packed LU record of C[J, E] per generation (lu_stride bytes,
    // layout bs_codegen._lu_solve_and_store) instead of coef_out / bound
    uint8_t* lu_out;
    uint32_t lu_stride;
    uint32_t grid_cap;   // k_decode_prepare_lu: max blocks (0 = one generation per wave)
    uint32_t lanes;      // 1: k_decode_prepare_lu_lanes (one generation per lane)
};
hipError_t launch_decode_prepare_cauchy(const PrepareCauchyArgs& a, hipStream_t st);

// Syndromes of codes without a syndrome kernel: gather the accepted sources
// (zero rows for erased ones) in source order, encode them with the
// bit-sliced encode kernels, XOR the accepted repair rows in.  Rows are read
// in whole 16-B units (Lu = ceil(L / 16)).
struct GatherArgs {
    const uint8_t* rows;   // received rows
    uint64_t rows_gen_stride, row_stride;
    const uint8_t* smap;   // [G][map_stride]: k source slots, r repair slots
    uint32_t map_stride;
    uint8_t* out;          // gather: sources [G][k]; xor: syndromes [G][r]
    uint64_t out_gen_stride, out_row_stride;
    uint32_t k, r, Lu, G;
    const uint64_t* rows_offs = nullptr;  // generation offset table of the received rows (nullptr: strided)
};
hipError_t launch_gather_sources(const GatherArgs& a, int num_cus, hipStream_t st);
hipError_t launch_xor_repairs(const GatherArgs& a, int num_cus, hipStream_t st);

// PD: prefetch depth in row pairs (V=1: 1..3, V=2: 1..2); k_pad must be a
// multiple of 2*(PD+1).
hipError_t launch_combine_uniform(const CombineUniformArgs& a, int R, int V, int PD, int num_cus,
                                  hipStream_t st);
hipError_t launch_combine_slots(const CombineSlotsArgs& a, int PD, int num_cus, hipStream_t st,
                                bool split_ok = true);
hipError_t launch_decode_prepare(const PrepareArgs& a, hipStream_t st);
size_t prepare_lds_bytes(uint32_t k, uint32_t e_max, uint32_t max_rows);
hipError_t launch_mul_slice(const uint8_t* a, const uint8_t* b, uint8_t* out, uint64_t n,
                            const uint8_t* explog, int num_cus, hipStream_t st);
hipError_t launch_fill_splitmix(uint8_t* dst, uint64_t n, uint64_t seed, uint64_t word_offset,
                                int num_cus, hipStream_t st);

// One encoder window of a multi-connection send batch: the window's ring at
// src + src_off (position i in slot (rot + i) % k), its repairs at
// rep + rep_off, rows rep_row_stride apart.
struct RingWin {
    uint64_t src_off, rep_off;
    uint32_t rot, L, src_row_stride, rep_row_stride;
};

// Small-batch encode (the per-packet send path: one or a few windows).
// repair[g][j] = sum_i coef[j*k + i] * src[g][i] over L bytes; lanes over
// (generation, repair, 16-B unit), units fastest.
struct EncodeSmallArgs {
    const uint8_t* src;
    uint64_t src_gen_stride, src_row_stride;
    uint8_t* rep;
    uint64_t rep_gen_stride, rep_row_stride;
    const uint8_t* coef;     // r x k device bytes
    const uint32_t* tab256;  // split-table records (8 dwords) of every coefficient
    uint32_t k, r, L, Lu, G;
    uint32_t rot;            // window row i is source row (i + rot) % k (a ring; 0: plain)
    const uint64_t* src_offs = nullptr;  // generation offset tables (nullptr: strided)
    const uint64_t* rep_offs = nullptr;
    // per-window records (nullptr: the scalar fields above); L / Lu above are
    // then the class maxima that size the tile grid
    const RingWin* wins = nullptr;
    // fused per-packet send (k_send_window): the ring slot of the new packet
    // and its 16-byte units (the packet itself travels in the arguments)
    uint8_t* fresh_dst = nullptr;
    uint32_t fresh_units = 0;
};

// Source packets of a send batch into their encoders' ring slots: bytes
// [0, len) from the staged copy at stage + src_off (zero padded to 16 bytes
// by the host), zeros to the slot's stride; dst2 (nullable) is the slot's
// twin in a double ring.
struct RingSlot {
    uint64_t src_off;
    uint8_t* dst;
    uint8_t* dst2;
    uint32_t len, stride;
};
hipError_t launch_ring_scatter(const uint8_t* stage, const RingSlot* slots, uint32_t M, hipStream_t st);

// Heterogeneous decode batches (qf_decode_batch_desc): a class's row indices
// gathered from the caller's arrays into [G][max_rows] (zero past n_rows)...
struct DescIndexArgs {
    const uint16_t* row_index;  // caller's row-index array
    const uint64_t* ri_off;     // [G] element offset of each generation's indices
    const uint32_t* n_rows;     // [G]
    uint16_t* out;              // [G][max_rows]
    uint32_t max_rows, G;
};
hipError_t launch_desc_gather_index(const DescIndexArgs& a, hipStream_t st);
// ... and its outputs scattered back: recovered indices to the caller's
// offsets, counts and statuses to the descriptors' positions
struct DescOutArgs {
    const uint16_t* rec_index_ws;  // [G][emax]
    const uint32_t* n_rec_ws;
    const int32_t* status_ws;
    const uint64_t* rec_index_off;  // [G]
    const uint32_t* desc_id;        // [G]
    uint16_t* rec_index;
    uint32_t* n_rec;
    int32_t* status;
    uint32_t emax, G;
};
hipError_t launch_desc_scatter_out(const DescOutArgs& a, hipStream_t st);

// base of generation g: base + offs[g] with an offset table, else base + g * stride
template <typename T>
__host__ __device__ inline T* gen_base(T* base, uint64_t g, uint64_t stride, const uint64_t* offs) {
    return base + (offs ? offs[g] : g * stride);
}
// Fused per-packet send: the new packet (pkt_bytes <= 16 fresh_units, in the
// kernel arguments) is window position k - 1 and goes into the ring slot
// a.fresh_dst; repairs to a.rep (host-coherent, whole 16-byte units).
constexpr uint32_t SEND_PKT_UNITS = 224;   // 3,584 bytes: with the arguments under 4 KiB
hipError_t launch_send_window(const EncodeSmallArgs& a, const uint8_t* pkt, uint32_t pkt_bytes, hipStream_t st);
hipError_t launch_encode_small(const EncodeSmallArgs& a, int num_cus, hipStream_t st);
// The same over per-window records (a.wins != nullptr), all repairs of a
// 64-unit tile per block (send batches of many windows).
hipError_t launch_encode_windows(const EncodeSmallArgs& a, int num_cus, hipStream_t st);

}  // namespace qf
