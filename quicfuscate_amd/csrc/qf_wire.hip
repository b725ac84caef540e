// qf_wire.hip -- wire framing on the device (encoder.rs:18-152), the step on
// either side of the codec kernels.
//
//   k_frame_batch   encode batch -> frames: source i "0x01 | payload",
//                   repair j "0x00 | k (BE u16) | C[j][0..k) | payload"
//   k_parse_frames  received frames -> decode-batch rows / row_index / n_rows
//
// Payloads sit at byte offset 1 or 3 + k inside a frame, so the copy loops
// move 16-byte blocks assembled from aligned dwords with v_alignbit (one
// block per lane); the header bytes and the ragged tail go byte by byte.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "qf_fec.h"

namespace {

#define QF_DEV __device__ __forceinline__

// bytes [off, off + 4) of a buffer read through aligned dwords
QF_DEV uint32_t load_u32_unaligned(const uint8_t* base, uint64_t off) {
    const uint64_t a = off & ~3ull;
    const uint32_t sh = (uint32_t)(off & 3) * 8;
    const uint32_t lo = *reinterpret_cast<const uint32_t*>(base + a);
    if (sh == 0) return lo;
    const uint32_t hi = *reinterpret_cast<const uint32_t*>(base + a + 4);
    return __builtin_amdgcn_alignbit(hi, lo, sh);
}

QF_DEV uint8_t cauchy_coeff(const uint8_t* sexp, const uint8_t* slog, uint32_t i, uint32_t k, uint32_t j) {
    const uint32_t d = (i & 0xFF) ^ ((k + j) & 0xFF);  // decoder.rs:280-298 (k + r <= 256: d != 0)
    return sexp[255 - slog[d]];
}

struct FrameArgs {
    const uint8_t* src;
    const uint8_t* rep;
    uint64_t src_row_stride, src_gen_stride, rep_row_stride, rep_gen_stride;
    uint8_t* frames;
    uint64_t frame_stride;
    uint32_t* frame_len;
    const uint8_t* explog;
    uint32_t k, r, L, blocks_per_frame;
    uint64_t total_blocks;
};

// one lane per 16-byte block of a frame (frames are frame_stride apart)
__global__ void __launch_bounds__(256) k_frame_batch(FrameArgs a) {
    __shared__ uint8_t sexp[512];
    __shared__ uint8_t slog[256];
    for (uint32_t i = threadIdx.x; i < 768; i += blockDim.x) {
        if (i < 512) sexp[i] = a.explog[i];
        else slog[i - 512] = a.explog[i];
    }
    __syncthreads();
    const uint32_t n = a.k + a.r;
    for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < a.total_blocks;
         b += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t f = b / a.blocks_per_frame;
        const uint32_t blk = (uint32_t)(b - f * a.blocks_per_frame);
        const uint64_t g = f / n;
        const uint32_t i = (uint32_t)(f - g * n);
        const bool sys = i < a.k;
        const uint32_t j = sys ? 0 : i - a.k;
        const uint32_t off = sys ? 1 : 3 + a.k;  // payload offset in the frame
        const uint32_t flen = off + a.L;
        const uint8_t* pay = sys ? a.src + g * a.src_gen_stride + (uint64_t)i * a.src_row_stride
                                 : a.rep + g * a.rep_gen_stride + (uint64_t)j * a.rep_row_stride;
        uint8_t* fr = a.frames + f * a.frame_stride;
        const uint32_t t0 = blk * 16;
        if (t0 >= flen) continue;
        if (blk == 0 && a.frame_len) a.frame_len[f] = flen;
        if (t0 >= off && t0 + 20 <= flen) {
            uint4 v;
            v.x = load_u32_unaligned(pay, t0 - off);
            v.y = load_u32_unaligned(pay, t0 - off + 4);
            v.z = load_u32_unaligned(pay, t0 - off + 8);
            v.w = load_u32_unaligned(pay, t0 - off + 12);
            *reinterpret_cast<uint4*>(fr + t0) = v;
        } else {
            for (uint32_t t = t0; t < t0 + 16 && t < flen; ++t) {
                uint8_t v;
                if (t >= off) v = pay[t - off];
                else if (t == 0) v = sys ? 1 : 0;
                else if (t == 1) v = (uint8_t)(a.k >> 8);
                else if (t == 2) v = (uint8_t)(a.k & 0xFF);
                else v = cauchy_coeff(sexp, slog, t - 3, a.k, j);
                fr[t] = v;
            }
        }
    }
}

struct ParseArgs {
    const uint8_t* frames;
    uint64_t frame_stride;
    const uint32_t* frame_len;
    const uint64_t* ids;
    const uint32_t* n_frames;
    uint8_t* rows;
    uint64_t row_stride, rows_gen_stride;
    uint16_t* row_index;
    uint32_t* n_rows;
    int32_t* frame_status;
    const uint8_t* explog;
    uint32_t k, r, L, max_rows;
};

// one 256-thread block per generation
__global__ void __launch_bounds__(256) k_parse_frames(ParseArgs a) {
    __shared__ uint8_t sexp[512];
    __shared__ uint8_t slog[256];
    __shared__ uint32_t slot_of[1024];   // frame -> output slot (or ~0)
    __shared__ uint32_t off_of[1024];    // payload offset of the frame
    __shared__ uint32_t len_of[1024];    // payload length
    __shared__ uint32_t wave_cnt[4];
    const uint32_t g = blockIdx.x;
    for (uint32_t i = threadIdx.x; i < 768; i += blockDim.x) {
        if (i < 512) sexp[i] = a.explog[i];
        else slog[i - 512] = a.explog[i];
    }
    __syncthreads();
    const uint32_t nf = a.n_frames ? min(a.n_frames[g], a.max_rows) : a.max_rows;
    uint32_t base = 0;
    for (uint32_t s0 = 0; s0 < nf; s0 += blockDim.x) {
        const uint32_t s = s0 + threadIdx.x;
        int32_t st = QF_OK;
        uint32_t idx = 0xFFFF, off = 0, plen = 0;
        if (s < nf) {
            const uint64_t fi = (uint64_t)g * a.max_rows + s;
            const uint8_t* fr = a.frames + fi * a.frame_stride;
            const uint32_t flen = a.frame_len[fi];
            if (flen == 0 || flen > a.frame_stride) {
                st = QF_EINVAL;  // "Raw data is empty"
            } else if (fr[0] == 1) {
                off = 1;
                idx = (uint32_t)(a.ids[fi] % a.k);  // decoder.rs:684
            } else if (flen < 3) {
                st = QF_ETOOSMALL;  // coefficient length missing (encoder.rs:33-38)
            } else {
                const uint32_t cl = ((uint32_t)fr[1] << 8) | fr[2];
                if (flen < 3 + cl) st = QF_ETOOSMALL;  // coefficients truncated
                else if (cl != a.k) st = QF_ERANGE;
                else {
                    // the coefficient vector must be Cauchy row j < r: c_0 = inv(k + j)
                    const uint32_t c0 = fr[3];
                    uint32_t j = 0xFFFF;
                    if (c0) j = ((uint32_t)sexp[255 - slog[c0]] - a.k) & 0xFF;
                    if (j >= a.r) st = QF_ERANGE;
                    else {
                        for (uint32_t i = 1; i < a.k && st == QF_OK; ++i)
                            if (fr[3 + i] != cauchy_coeff(sexp, slog, i, a.k, j)) st = QF_ERANGE;
                    }
                    off = 3 + cl;
                    idx = a.k + j;
                }
            }
            if (st == QF_OK) {
                plen = flen - off;
                if (plen > a.L) st = QF_EINVAL;
            }
            a.frame_status[fi] = st;
        }
        const bool ok = s < nf && st == QF_OK;
        // block-wide exclusive prefix of ok (4 waves)
        const uint64_t bal = __ballot(ok);
        const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        const uint32_t before = __popcll(bal & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
        if (lane == 0) wave_cnt[w] = __popcll(bal);
        __syncthreads();
        uint32_t woff = 0;
        for (uint32_t q = 0; q < w; ++q) woff += wave_cnt[q];
        uint32_t total = 0;
        for (uint32_t q = 0; q < 4; ++q) total += wave_cnt[q];
        if (s < nf && s < 1024) {
            slot_of[s] = ok ? base + woff + before : 0xFFFFFFFFu;
            off_of[s] = off;
            len_of[s] = plen;
        }
        if (ok) a.row_index[(uint64_t)g * a.max_rows + base + woff + before] = (uint16_t)idx;
        base += total;
        __syncthreads();
    }
    if (threadIdx.x == 0 && a.n_rows) a.n_rows[g] = base;
    __syncthreads();
    // payload copy: 16-byte blocks of every accepted row, zero beyond the payload
    const uint32_t bpr = (a.L + 15) / 16;
    const uint32_t nwork = min(nf, 1024u) * bpr;
    for (uint32_t w = threadIdx.x; w < nwork; w += blockDim.x) {
        const uint32_t s = w / bpr, blk = w - s * bpr;
        const uint32_t slot = slot_of[s];
        if (slot == 0xFFFFFFFFu) continue;
        const uint64_t fi = (uint64_t)g * a.max_rows + s;
        const uint8_t* src = a.frames + fi * a.frame_stride + off_of[s];
        uint8_t* dst = a.rows + g * a.rows_gen_stride + (uint64_t)slot * a.row_stride;
        const uint32_t t0 = blk * 16, plen = len_of[s];
        if (t0 + 20 <= plen) {
            const uint64_t o = (uint64_t)(src - a.frames);
            uint4 v;
            v.x = load_u32_unaligned(a.frames, o + t0);
            v.y = load_u32_unaligned(a.frames, o + t0 + 4);
            v.z = load_u32_unaligned(a.frames, o + t0 + 8);
            v.w = load_u32_unaligned(a.frames, o + t0 + 12);
            *reinterpret_cast<uint4*>(dst + t0) = v;
        } else {
            for (uint32_t t = t0; t < t0 + 16 && t < a.L; ++t) dst[t] = t < plen ? src[t] : 0;
        }
    }
}

}  // namespace

namespace qf {

hipError_t launch_frame_batch(const uint8_t* src, const uint8_t* rep, const qf_encode_shape& sh, uint32_t G,
                              uint8_t* frames, uint64_t frame_stride, uint32_t* frame_len,
                              const uint8_t* explog, int num_cus, hipStream_t st) {
    FrameArgs a{};
    a.src = src;
    a.rep = rep;
    a.src_row_stride = sh.src_row_stride;
    a.src_gen_stride = sh.src_gen_stride;
    a.rep_row_stride = sh.rep_row_stride;
    a.rep_gen_stride = sh.rep_gen_stride;
    a.frames = frames;
    a.frame_stride = frame_stride;
    a.frame_len = frame_len;
    a.explog = explog;
    a.k = sh.k;
    a.r = sh.r;
    a.L = sh.L;
    a.blocks_per_frame = (uint32_t)((3 + sh.k + sh.L + 15) / 16);
    a.total_blocks = (uint64_t)G * (sh.k + sh.r) * a.blocks_per_frame;
    if (a.total_blocks == 0) return hipSuccess;
    uint64_t blocks = (a.total_blocks + 255) / 256;
    const uint64_t cap = (uint64_t)num_cus * 8;
    if (blocks > cap) blocks = cap;
    hipLaunchKernelGGL(k_frame_batch, dim3((uint32_t)blocks), dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_parse_frames(const uint8_t* frames, uint64_t frame_stride, const uint32_t* frame_len,
                               const uint64_t* ids, const uint32_t* n_frames, uint32_t k, uint32_t r, uint32_t L,
                               uint32_t G, uint32_t max_rows, uint8_t* rows, uint64_t row_stride,
                               uint64_t rows_gen_stride, uint16_t* row_index, uint32_t* n_rows,
                               int32_t* frame_status, const uint8_t* explog, hipStream_t st) {
    ParseArgs a{};
    a.frames = frames;
    a.frame_stride = frame_stride;
    a.frame_len = frame_len;
    a.ids = ids;
    a.n_frames = n_frames;
    a.rows = rows;
    a.row_stride = row_stride;
    a.rows_gen_stride = rows_gen_stride;
    a.row_index = row_index;
    a.n_rows = n_rows;
    a.frame_status = frame_status;
    a.explog = explog;
    a.k = k;
    a.r = r;
    a.L = L;
    a.max_rows = max_rows;
    if (G == 0) return hipSuccess;
    hipLaunchKernelGGL(k_parse_frames, dim3(G), dim3(256), 0, st, a);
    return hipGetLastError();
}

}  // namespace qf
