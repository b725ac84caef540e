// qf_bs.hip -- loader / launcher of the bit-sliced Cauchy encode kernels.
//
// The kernels are generated gfx950 assembly (quicfuscate_amd/bs_codegen.py):
// multiplication by each coefficient of the reference's fixed Cauchy matrix
// (decoder.rs:280-298) is specialised into straight-line full-rate v_xor_b32
// over bit-planes.  build_lib.py assembles them and embeds the code objects
// (qf_bs_blobs.inc); this file loads them into the context's device with
// hipModuleLoadData and launches them with a packed kernarg buffer.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include <mutex>

#include "qf_bs.h"
#include "qf_fec.h"
#include "qf_internal.h"

struct QfBsEntry {
    uint32_t k, r, pd;
    uint32_t rt, j0;  // enc passes: repairs j0 .. j0 + r - 1 of the (k, rt) code
    char mode;  // 'e' encode, 'E' additive-FFT encode, 'g' sliding-window encode, 'C' additive-FFT chunked decode, 's' decode syndromes, 'w' syndromes (scalar slot map), 'd'/'c' fused decode,
                // 'k' the chunked fused decode with an item's rows split over its workgroup's 4 waves,
                // 'f' the encode (passes of C5 codes) with an item's sources split the same way,
                // 'M' / 'N' every encode pass of a code in one dispatch (plain / additive-FFT passes),
                // 'X' / 'Y' every 'w' pass in one pass-major dispatch (plain / additive-FFT passes)
                // 'Z' the additive-FFT 'w' passes item-major, one wave per pass, row work shared in LDS
    uint32_t map_stride;
    const char* name;
    const unsigned char* data;  // the code object, zlib-compressed (build_lib.py)
    size_t size;                // its size inflated
    uint32_t waves;  // waves per workgroup ('M' / 'N': one per pass, each on the workgroup's item)
    uint32_t passes; // 'X': passes laid out pass-major over the grid (workgroup ranges of equal size)
    size_t zsize;    // bytes at data
};
#include "qf_bs_blobs.inc"

namespace qf {

// The inflated code object of a table entry: inflated once per process and
// kept (contexts on several devices load the same image).
static const void* blob_image(const QfBsEntry* e) {
    static std::mutex mu;
    static unsigned char* images[sizeof(qf_bs_table) / sizeof(qf_bs_table[0])] = {};
    const size_t idx = (size_t)(e - qf_bs_table);
    std::lock_guard<std::mutex> g(mu);
    if (!images[idx]) {
        unsigned char* buf = static_cast<unsigned char*>(malloc(e->size));
        uLongf n = (uLongf)e->size;
        if (!buf) return nullptr;
        if (uncompress(buf, &n, e->data, (uLong)e->zsize) != Z_OK || n != e->size) {
            free(buf);
            return nullptr;
        }
        images[idx] = buf;
    }
    return images[idx];
}

static hipError_t load_module(BsCache& cache, int idx, const QfBsEntry* e) {
    const void* image = blob_image(e);
    if (!image) {
        note_launch_refused("qf_bs.hip code object inflate", __LINE__);
        return hipErrorInvalidImage;
    }
    hipError_t err = hipModuleLoadData(&cache.mod[idx], image);
    if (err == hipSuccess) err = hipModuleGetFunction(&cache.fn[idx], cache.mod[idx], e->name);
    if (err != hipSuccess && getenv("QF_BS_DEBUG")) fprintf(stderr, "%s: module load %d\n", e->name, (int)err);
    return err;
}

// QF_BS_DEBUG=1: name the check behind a hipErrorInvalidValue on stderr
// (qf_last_error carries the refusal's line whether or not it is set)
static hipError_t bs_invalid(int line) {
    static const bool on = getenv("QF_BS_DEBUG") != nullptr;
    if (on) fprintf(stderr, "qf_bs.hip:%d: launch refused\n", line);
    note_launch_refused("qf_bs.hip", line);
    return hipErrorInvalidValue;
}

// the kernel (first pass, j0 = 0) of the (k, r) code
static const QfBsEntry* find(char mode, uint32_t k, uint32_t r) {
    for (const auto& e : qf_bs_table)
        if (e.mode == mode && e.k == k && e.rt == r && e.j0 == 0) return &e;
    return nullptr;
}

bool bs_available(uint32_t k, uint32_t r) { return find('e', k, r) != nullptr; }
bool synw_available(uint32_t k, uint32_t r) { return find('w', k, r) != nullptr; }
bool syn_available(uint32_t k, uint32_t r) { return find('s', k, r) != nullptr; }

const char* bs_name(uint32_t k, uint32_t r, bool fft) {
    const QfBsEntry* e = fft ? find('E', k, r) : nullptr;
    if (!e) e = find('e', k, r);
    return e ? e->name : nullptr;
}

const char* syn_name(uint32_t k, uint32_t r) {
    const QfBsEntry* e = find('s', k, r);
    return e ? e->name : nullptr;
}

uint32_t syn_map_stride(uint32_t k, uint32_t r) {
    const QfBsEntry* e = find('s', k, r);
    return e ? e->map_stride : 0;
}

static void magic_for(uint32_t U, uint32_t* magic, uint32_t* shift) {
    uint32_t s = 0;
    while ((1u << s) < U) ++s;  // 2^(s-1) < U <= 2^s
    const uint64_t num = 1ull << (31 + s);
    *magic = (uint32_t)((num + U - 1) / U);
    *shift = s - 1;
}

// Shared launch: kernarg words as bs_codegen.kernargs (80 bytes).  Items of
// 128 16-byte units, one wave per item (non-persistent grid: staggered wave
// start-up overlaps one wave's loads with another's XOR work).
// Lv: lane units per row (>= L/16); s19: enc = units stored per row, syn =
// slot-map stride (bs_codegen.py kernarg layout).
static hipError_t launch(BsCache& cache, const QfBsEntry* e, int num_cus, hipStream_t st,
                         const uint8_t* src, uint8_t* dst, uint64_t sgs, uint64_t dgs, uint64_t srs,
                         uint64_t drs, uint32_t L, uint32_t G, uint32_t Lv, uint32_t s19,
                         const uint8_t* smap, const uint8_t* zero, const uint8_t* lu = nullptr,
                         uint32_t lu_stride = 0, const uint32_t* tab256 = nullptr,
                         const uint64_t* src_offs = nullptr, const uint64_t* dst_offs = nullptr,
                         const uint32_t* bound = nullptr) {
    if (!e) return bs_invalid(__LINE__);
    int idx = (int)(e - qf_bs_table);
    if (idx >= BsCache::kMax) return bs_invalid(__LINE__);
    // a partial last unit: enc in the zero-tail lane space (its bytes >= L are
    // masked to zero before the store); syn (the syndrome rows' tail is junk
    // the combine never stores); the lane-chunk decode ('c': the lane holding
    // the last unit stores it bytewise); never the item-layout decode ('d')
    const bool chunked = e->mode == 'c' || e->mode == 'k' || e->mode == 'C';
    const bool merged = e->mode == 'M' || e->mode == 'N' || e->mode == 'Z';
    // (every encoder letter: the kernarg words 16..19 are its tail byte masks)
    const bool enc = e->mode == 'e' || e->mode == 'f' || e->mode == 'E' || e->mode == 'M' || e->mode == 'N' ||
                     e->mode == 'g';
    if ((L % 16 && (e->mode == 'd' || (enc && Lv != s19))) || L < 32 ||
        sgs >= (1ull << 32) || dgs >= (1ull << 32) ||
        srs >= (1ull << 32) || drs >= (1ull << 32))
        return bs_invalid(__LINE__);
    if (!cache.fn[idx]) {
        hipError_t err = load_module(cache, idx, e);
        if (err != hipSuccess) return err;
    }
    const uint32_t Lu = (L + 15) / 16;
    // lane-chunk layout of the chunked fused decode ('c'): lane-chunk = units
    // q and q + Q of one generation, Q = ceil(Lu / 2), 64 lane-chunks per item
    if (chunked) Lv = (Lu + 1) / 2;
    else if (Lv < Lu) return bs_invalid(__LINE__);
    if (Lv < 2) return bs_invalid(__LINE__);
    const uint64_t total = (uint64_t)G * Lv;
    if (total >= (1ull << 31)) return bs_invalid(__LINE__);
    uint32_t magic, shift;
    magic_for(Lv, &magic, &shift);
    const uint32_t n_items = (uint32_t)(chunked ? (total + 63) / 64 : (total + 127) / 128);
    // 'k' / 'f' / merged passes: one workgroup per item
    const bool wg_item = e->mode == 'k' || e->mode == 'f' || merged;
    uint32_t blocks = wg_item ? n_items : (n_items + 3) / 4;
    if (blocks == 0) return hipSuccess;
    // persistent grids (the item loop strides by the grid's wave count):
    // QF_ENC_BLOCKS_PER_CU / QF_DEC_BLOCKS_PER_CU cap the grid at that many
    // 4-wave blocks per CU, so an encode and a decode launched on two streams
    // can be resident on every SIMD at once
    {
        const int c = (int)cache.get(enc ? QF_OPT_ENC_BLOCKS_PER_CU : QF_OPT_DEC_BLOCKS_PER_CU);
        // (a block of the merged kernels is one item's passes: up to 4 per CU fill it)
        const uint32_t cap = (uint32_t)(c * num_cus) * (merged ? 4u / e->waves : 1u);
        if (c > 0 && num_cus > 0 && blocks > cap) blocks = cap;
    }
    uint32_t a[32] = {};
    a[0] = (uint32_t)(uintptr_t)src;
    a[1] = (uint32_t)((uintptr_t)src >> 32);
    a[2] = (uint32_t)(uintptr_t)dst;
    a[3] = (uint32_t)((uintptr_t)dst >> 32);
    a[4] = (uint32_t)sgs;
    a[5] = (uint32_t)dgs;
    a[6] = (uint32_t)srs;
    a[7] = (uint32_t)drs;
    a[8] = Lu;
    a[9] = Lv;
    a[10] = (uint32_t)total;
    a[11] = magic;
    a[12] = shift;
    a[13] = n_items;
    a[14] = merged ? blocks : blocks * 4;   // item stride: workgroups (merged) or waves
    a[15] = s19;
    if (enc) {
        // byte masks of the last unit's dwords (bs_codegen.tail_masks)
        const uint32_t tb = L % 16 ? L % 16 : 16;
        for (uint32_t d = 0; d < 4; ++d) {
            const int32_t valid = (int32_t)tb - 4 * (int32_t)d;
            a[16 + d] = valid >= 4 ? 0xFFFFFFFFu : (valid <= 0 ? 0u : (1u << (8 * valid)) - 1);
        }
    } else {
        a[16] = (uint32_t)(uintptr_t)smap;
        a[17] = (uint32_t)((uintptr_t)smap >> 32);
        a[18] = (uint32_t)(uintptr_t)zero;
        a[19] = (uint32_t)((uintptr_t)zero >> 32);
    }
    a[20] = (uint32_t)(uintptr_t)lu;
    a[21] = (uint32_t)((uintptr_t)lu >> 32);
    a[22] = lu_stride;
    if (chunked) a[23] = L % 16;   // bytes of the partial last unit (0: whole)
    a[24] = (uint32_t)(uintptr_t)tab256;
    a[25] = (uint32_t)((uintptr_t)tab256 >> 32);
    // generation offset tables, the last 16 kernarg bytes (bs_codegen S_OFFS)
    const int ot = (e->mode == 'd' || chunked) ? 28 : 20;
    a[ot] = (uint32_t)(uintptr_t)src_offs;
    a[ot + 1] = (uint32_t)((uintptr_t)src_offs >> 32);
    a[ot + 2] = (uint32_t)(uintptr_t)dst_offs;
    a[ot + 3] = (uint32_t)((uintptr_t)dst_offs >> 32);
    size_t sz = (size_t)(ot + 4) * 4;
    if (e->mode == 'w' || e->mode == 'X' || e->mode == 'Y' || e->mode == 'Z') {   // per-generation pass bound (KERNARG_BYTES_SYNW)
        a[24] = (uint32_t)(uintptr_t)bound;
        a[25] = (uint32_t)((uintptr_t)bound >> 32);
        sz = 26 * 4;
    }
    void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz,
                   HIP_LAUNCH_PARAM_END};
    // 'X': the grid holds every pass's `blocks` workgroups, pass-major
    const uint32_t grid = blocks * (e->mode == 'X' || e->mode == 'Y' ? e->passes : 1u);
    const hipError_t err = hipModuleLaunchKernel(cache.fn[idx], grid, 1, 1, 64 * e->waves, 1, 1, 0, st, nullptr, cfg);
    if (err != hipSuccess && getenv("QF_BS_DEBUG"))
        fprintf(stderr, "%s: hipModuleLaunchKernel %d (%u blocks x %u)\n", e->name, (int)err, blocks, 64 * e->waves);
    return err;
}

uint32_t bs_padded_units(uint32_t L) { return ((L + 15) / 16 + 7) / 8 * 8; }

bool bs_zero_tail_fits(uint32_t r, uint32_t L, uint64_t drs, uint64_t dgs) {
    const uint64_t row = 16ull * bs_padded_units(L);
    return (r == 1 || drs >= row) && dgs >= (uint64_t)(r - 1) * drs + row;
}

hipError_t bs_launch(BsCache& cache, int num_cus, hipStream_t st, uint32_t k, uint32_t r,
                     const uint8_t* src, uint8_t* dst, uint64_t sgs, uint64_t dgs, uint64_t srs,
                     uint64_t drs, uint32_t L, uint32_t G, bool zero_tail, const uint64_t* src_offs,
                     const uint64_t* dst_offs, const char** name_out) {
    // zero tail: lane space padded to whole 128-B lines per row and the tail
    // [L, 16 Lv) of every repair row written with zeros, so every line the
    // kernel stores is whole (tools/bs_lab.py: partial lines shared by two
    // waves cut the write rate from ~5.7 to ~4 TB/s at L = 1200)
    const uint32_t Lu = L / 16;
    const uint32_t Lv = zero_tail ? bs_padded_units(L) : Lu;
    // (with a destination offset table each generation's repair block is the
    // caller's: only the row stride is checked here)
    if (zero_tail && !(dst_offs ? (r == 1 || drs >= 16ull * bs_padded_units(L)) : bs_zero_tail_fits(r, L, drs, dgs)))
        return bs_invalid(__LINE__);
    if (!zero_tail && L % 16) return bs_invalid(__LINE__);
    if (!find('e', k, r)) return bs_invalid(__LINE__);
    // batches of at most one item (128 units) per CU take the 'f' kernels
    // (the sources of an item split over its workgroup's four waves) where
    // they exist, unless QF_ENCODE_KSPLIT=0
    char mode = 'e';
    {
        const uint64_t items = ((uint64_t)G * Lv + 127) / 128;
        const bool fft = cache.get(QF_OPT_FFT_KERNELS);
        if (cache.get(QF_OPT_ENCODE_KSPLIT) && find('f', k, r) && num_cus > 0 && items <= (uint64_t)num_cus) mode = 'f';
        else if (cache.get(QF_OPT_ENCODE_MERGED) && fft && find('N', k, r)) mode = 'N';
        else if (cache.get(QF_OPT_ENCODE_MERGED) && find('M', k, r)) mode = 'M';
        else if (fft && find('E', k, r)) mode = 'E';
        // overlapping generations (sliding windows: generation stride below k
        // row strides) take the shape's 'g' kernel where one is built
        // (QF_SLIDING_KERNELS): cached row loads, since the next windows read
        // the same rows, and for (48, 8) the hybrid FFT pass
        if (mode != 'f' && cache.get(QF_OPT_SLIDING_KERNELS) && !src_offs && sgs < (uint64_t)k * srs &&
            find('g', k, r))
            mode = 'g';
    }
    // one launch per pass of repairs (codes with more repairs than a kernel
    // holds): pass j0 writes repair rows j0 .. j0 + r_pass - 1
    for (const auto& e : qf_bs_table) {
        if (e.mode != mode || e.k != k || e.rt != r) continue;
        if (name_out && e.j0 == 0) *name_out = e.name;
        hipError_t err = launch(cache, &e, num_cus, st, src, dst + (uint64_t)e.j0 * drs, sgs, dgs, srs, drs, L, G,
                                Lv, Lv, nullptr, nullptr, nullptr, 0, nullptr, src_offs, dst_offs);
        if (err != hipSuccess) return err;
    }
    return hipSuccess;
}

hipError_t syn_launch(BsCache& cache, int num_cus, hipStream_t st, uint32_t k, uint32_t r,
                      const uint8_t* rows, uint8_t* syn, uint64_t rgs, uint64_t sgs, uint64_t rs,
                      uint64_t srs, uint32_t L, uint32_t G, const uint8_t* smap, uint32_t map_stride,
                      const uint8_t* zero, const uint64_t* rows_offs) {
    const QfBsEntry* e = find('s', k, r);
    if (!e || map_stride != e->map_stride || !zero) return bs_invalid(__LINE__);
    // syndrome rows live in the library's workspace: always the padded lane
    // space (srs >= 16 * bs_padded_units(L); the tail holds junk)
    const uint32_t Lv = bs_padded_units(L);
    if (srs < 16ull * Lv) return bs_invalid(__LINE__);
    return launch(cache, e, num_cus, st, rows, syn, rgs, sgs, rs, srs, L, G, Lv, map_stride, smap, zero, nullptr, 0,
                  nullptr, rows_offs, nullptr);
}

hipError_t synw_launch(BsCache& cache, int num_cus, hipStream_t st, uint32_t k, uint32_t r,
                       const uint8_t* rows, uint8_t* syn, uint64_t rgs, uint64_t sgs, uint64_t rs,
                       uint64_t srs, uint32_t L, uint32_t G, const uint8_t* smap, uint32_t map_stride,
                       const uint8_t* zero, const uint32_t* bound, const uint64_t* rows_offs) {
    const QfBsEntry* first = find('w', k, r);
    if (!first || map_stride != first->map_stride || !zero) return bs_invalid(__LINE__);
    // an item (128 units) must lie in at most two generations
    const uint32_t Lv = bs_padded_units(L);
    if (Lv < 128 || srs < 16ull * Lv) return bs_invalid(__LINE__);
    // the passes in one dispatch unless QF_ENCODE_MERGED=0: the additive-FFT
    // ones item-major with the row work shared in LDS ('Z', QF_SYNW_SHARED) or
    // pass-major ('Y') unless QF_FFT_KERNELS=0, else the plain ones ('X')
    const bool merged = cache.get(QF_OPT_ENCODE_MERGED);
    const bool fft = merged && cache.get(QF_OPT_FFT_KERNELS);
    const char mode = fft && cache.get(QF_OPT_SYNW_SHARED) && find('Z', k, r) ? 'Z'
                      : fft && find('Y', k, r) ? 'Y'
                      : merged && find('X', k, r) ? 'X' : 'w';
    for (const auto& e : qf_bs_table) {
        if (e.mode != mode || e.k != k || e.rt != r) continue;
        // every pass of the chosen mode reads the slot map at the caller's
        // stride (checked per entry: 'X' / 'Y' / 'Z' are separate specs)
        if (e.map_stride != map_stride) return bs_invalid(__LINE__);
        hipError_t err = launch(cache, &e, num_cus, st, rows, syn + (uint64_t)e.j0 * srs, rgs, sgs, rs, srs, L, G, Lv,
                                map_stride, smap, zero, nullptr, 0, nullptr, rows_offs, nullptr, bound);
        if (err != hipSuccess) return err;
    }
    return hipSuccess;
}

// the chunked fused decode unless QF_DECODE_LEGACY=1 (or the row is too short
// for two units per lane-chunk pair); for a batch of at most one item per CU
// (G > 0 and num_cus given) its row-split form 'k', unless QF_DECODE_KSPLIT=0
// (tools/dec_lab.py --small: 32 against 51-56 us from G = 1 to 256 at the C3
// shape; past one item per CU the one-wave-per-item kernel wins)
static const QfBsEntry* find_dec(const BsCache* cache, uint32_t k, uint32_t r, uint32_t L, uint32_t G = 0,
                                 int num_cus = 0) {
    const bool legacy = cache && cache->get(QF_OPT_DECODE_PATH) == 2;
    const bool fft = cache && cache->get(QF_OPT_FFT_KERNELS);
    const QfBsEntry* c = find('c', k, r);
    if (c && !legacy && (L == 0 || (L + 15) / 16 >= 3)) {
        if (G && num_cus > 0 && L) {
            const bool ks = !cache || cache->get(QF_OPT_DECODE_KSPLIT);
            const uint64_t Q = ((L + 15) / 16 + 1) / 2, items = ((uint64_t)G * Q + 63) / 64;
            const QfBsEntry* kk = find('k', k, r);
            if (ks && kk && items <= (uint64_t)num_cus) return kk;
        }
        if (fft) {
            const QfBsEntry* cf = find('C', k, r);
            if (cf) return cf;
        }
        return c;
    }
    return find('d', k, r);
}

bool dec_available(uint32_t k, uint32_t r) { return find_dec(nullptr, k, r, 0) != nullptr; }

const char* dec_name(const BsCache* cache, uint32_t k, uint32_t r, uint32_t L, uint32_t G, int num_cus) {
    const QfBsEntry* e = find_dec(cache, k, r, L, G, num_cus);
    return e ? e->name : nullptr;
}

hipError_t dec_launch(BsCache& cache, int num_cus, hipStream_t st, uint32_t k, uint32_t r,
                      const uint8_t* rows, uint8_t* rec, uint64_t rgs, uint64_t rec_gs, uint64_t rs,
                      uint64_t rec_rs, uint32_t L, uint32_t G, const uint8_t* smap, uint32_t map_stride,
                      const uint8_t* zero, const uint8_t* lu, uint32_t lu_stride, const uint32_t* tab256,
                      const uint64_t* rows_offs, const uint64_t* rec_offs) {
    const QfBsEntry* e = find_dec(&cache, k, r, L, G, num_cus);
    if (!e || map_stride != e->map_stride || !zero || !lu || !tab256 || (lu_stride & 15) || lu_stride < 272)
        return bs_invalid(__LINE__);
    // the LU record pointer is computed with a 32-bit stride multiply
    if ((uint64_t)G * lu_stride >= (1ull << 40)) return bs_invalid(__LINE__);
    // unpadded lane space: the kernel is VALU-bound, padding lanes would be
    // pure extra work (and the recovered rows are caller memory, payload only)
    if (L % 16 && e->mode != 'c' && e->mode != 'k' && e->mode != 'C') return bs_invalid(__LINE__);
    return launch(cache, e, num_cus, st, rows, rec, rgs, rec_gs, rs, rec_rs, L, G, (L + 15) / 16, map_stride, smap, zero,
                  lu, lu_stride, tab256, rows_offs, rec_offs);
}

// Bit-sliced payload pass (bs_codegen.py "cmb", mode 'm'): one generation
// per item, wave-uniform coefficients (kernarg layout: bs_codegen.cmb_kernargs)
bool cmb_available() { return find('m', 0, 16) != nullptr; }
bool cmb_pass_major_available() { return find('P', 0, 16) != nullptr; }
// the payload kernel of a launch: single (16 outputs, 'm'), wide (24, 'm'
// r = 24), pass-major ('P') or the pass-major item-major interleave ('Q',
// QF_COMBINE_XCD: workgroup w runs pass (w >> 3) mod P for slot
// 8 ((w >> 3) div P) + w % 8, so the P passes of a slot are neighbours on one
// XCD); each with its products as calls into per-coefficient code blocks
// ('j' / 'j' / 'J' / 'V', QF_COMBINE_JUMP) where built
static const QfBsEntry* cmb_pick(BsCache& cache, char plain, char jump, uint32_t r) {
    const QfBsEntry* j = cache.get(QF_OPT_COMBINE_JUMP) ? find(jump, 0, r) : nullptr;
    return j ? j : find(plain, 0, r);
}

// the 24-output pass-major launch ('W', jump products, QF_COMBINE_PM24) for
// 4 record passes (e_max 49-64): 3 passes of 24 instead of 4 of 16, the
// records' pass stride plus one piece (8 B) in 32 bits.  At e_max 33-48 the
// generations' own e usually needs two passes either way, and there the
// 24-output form measured 2-3 % slower (DESIGN 3.7 "Round 6")
static bool cmb_pm24_ok(BsCache& cache, const CombineSlotsArgs& a, uint32_t passes, uint64_t pass_stride,
                        uint32_t e_max) {
    return passes == 4 && passes <= kCmbMaxPasses && e_max > 48 && e_max <= 64 && a.pass == 0 &&
           pass_stride + 8 < (1ull << 32) && 72ull * a.dst_row_stride < (1ull << 32) &&
           cache.get(QF_OPT_COMBINE_JUMP) && cache.get(QF_OPT_COMBINE_PM24) && find('W', 0, 24) != nullptr;
}

static const QfBsEntry* cmb_entry(BsCache& cache, bool wide, uint32_t passes, bool pm24 = false) {
    if (pm24) return find('W', 0, 24);
    if (wide) return cmb_pick(cache, 'm', 'j', 24);
    if (passes <= 1) return cmb_pick(cache, 'm', 'j', 16);
    if (cache.get(QF_OPT_COMBINE_XCD) && passes <= 4) {
        const QfBsEntry* q = cmb_pick(cache, 'Q', 'V', 16);
        if (q) return q;
    }
    return cmb_pick(cache, 'P', 'J', 16);
}

const char* cmb_kernel_name(BsCache& cache, const CombineSlotsArgs& a, uint32_t passes, uint64_t pass_stride,
                            uint32_t e_max) {
    const QfBsEntry* e = cmb_entry(cache, cmb_wide_ok(cache, a, passes, pass_stride, e_max), passes,
                                   cmb_pm24_ok(cache, a, passes, pass_stride, e_max));
    return e ? e->name : "qf_combine_bs?";
}

bool cmb_pass_major_ok(uint32_t passes, uint64_t dst_row_stride, uint64_t pass_stride) {
    return passes > 1 && passes <= kCmbMaxPasses && pass_stride < (1ull << 32) &&
           16ull * (passes - 1) * dst_row_stride < (1ull << 32) && cmb_pass_major_available();
}

bool cmb_wide_ok(BsCache& cache, const CombineSlotsArgs& a, uint32_t passes, uint64_t pass_stride,
                 uint32_t e_max) {
    return passes == 2 && e_max > 16 && e_max <= 24 && a.pass == 0 && pass_stride < (1ull << 32) &&
           24ull * a.dst_row_stride < (1ull << 32) && cache.get(QF_OPT_COMBINE_WIDE) && find('m', 0, 24) != nullptr;
}

// kernarg word 33 of the interleaved pass-major kernel (bs_codegen.pm_xcd_word):
// (ceil(2^16 / P) << 3) | P, the kernel's h div P by multiply and shift
static uint32_t pm_xcd_word(uint32_t passes) { return ((65536u + passes - 1) / passes) << 3 | passes; }

hipError_t cmb_launch(BsCache& cache, int num_cus, hipStream_t st, const CombineSlotsArgs& a,
                      const uint32_t* idxtab, uint32_t passes, uint64_t pass_stride, uint32_t e_max) {
    // the wide pass: 24 outputs per item (192 accumulator VGPRs, still two
    // waves per SIMD), outputs 16..23 from the row's pass-1 record, so a
    // batch of 17-24 outputs reads and transposes each input row once
    // instead of once per 16-output pass (output j's row at j * dst stride:
    // a 32-bit product in the kernel)
    const bool wide = cmb_wide_ok(cache, a, passes, pass_stride, e_max);
    const bool pm24 = !wide && cmb_pm24_ok(cache, a, passes, pass_stride, e_max);
    const QfBsEntry* e = cmb_entry(cache, wide, passes, pm24);
    const bool xcd = e && (e->mode == 'Q' || e->mode == 'V');
    const uint32_t launch_passes = pm24 ? (e_max + 23) / 24 : wide ? 1 : passes;
    if (!e || !idxtab || a.L == 0 || a.row_stride >= (1ull << 32) || 16ull * a.dst_row_stride >= (1ull << 32) ||
        a.coef_gen_stride >= (1ull << 32) || passes == 0 || (passes > 1 && a.pass != 0) ||
        (passes > 1 && !wide && !cmb_pass_major_ok(passes, a.dst_row_stride, pass_stride)))
        return bs_invalid(__LINE__);
    const int idx = (int)(e - qf_bs_table);
    if (idx >= BsCache::kMax) return bs_invalid(__LINE__);
    if (!cache.fn[idx]) {
        hipError_t err = load_module(cache, idx, e);
        if (err != hipSuccess) return err;
    }
    const uint32_t Lu = (a.L + 15) / 16, Q = (Lu + 1) / 2, ipg = (Q + 63) / 64;
    const uint64_t G = a.total_units / Lu;
    const uint64_t n_items = G * ipg;
    if (n_items == 0) return hipSuccess;
    if (n_items >= (1ull << 31)) return bs_invalid(__LINE__);
    uint32_t magic = 0, shift = 0;
    if (ipg >= 2) magic_for(ipg, &magic, &shift);
    // persistent grid: two 4-wave blocks per CU (192 VGPRs: two waves per SIMD)
    uint64_t blocks = (n_items + 3) / 4;
    const uint64_t cap = (uint64_t)(num_cus > 0 ? num_cus : 256) * 2;
    if (blocks > cap) blocks = cap;
    if (xcd) blocks = (blocks + 7) / 8 * 8;   // slots in groups of 8, one per XCD: a grid of 8 P-blocks
    auto lo = [](const void* p) { return (uint32_t)(uintptr_t)p; };
    auto hi = [](const void* p) { return (uint32_t)((uintptr_t)p >> 32); };
    uint32_t w[34] = {lo(a.rows), hi(a.rows), lo(a.dst), hi(a.dst),
                      (uint32_t)a.rows_gen_stride, (uint32_t)(a.rows_gen_stride >> 32),
                      (uint32_t)a.dst_gen_stride, (uint32_t)(a.dst_gen_stride >> 32),
                      (uint32_t)a.row_stride, (uint32_t)a.dst_row_stride, lo(a.coef), hi(a.coef),
                      (uint32_t)a.coef_gen_stride, a.pass, lo(a.n_out), hi(a.n_out), lo(a.bound), hi(a.bound),
                      lo(idxtab), hi(idxtab), lo(a.rows_offs), hi(a.rows_offs), lo(a.dst_offs), hi(a.dst_offs),
                      a.L, Lu, Q, ipg, (uint32_t)n_items, (uint32_t)blocks * 4, magic, shift,
                      (uint32_t)pass_stride, xcd ? pm_xcd_word(passes) : pm24 ? passes : 0u};
    // (pass-major: word 32 = the records' pass stride; the grid holds every
    // pass's `blocks` workgroups, pass p's at [p blocks, (p + 1) blocks), or
    // interleaved ('Q': word 33 = pm_xcd_word(passes)))
    // (the wide pass: word 32 too, one pass's grid)
    size_t sz = passes > 1 ? sizeof(w) : 32 * sizeof(uint32_t);
    void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, w, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
    return hipModuleLaunchKernel(cache.fn[idx], (uint32_t)blocks * launch_passes, 1, 1, 256, 1, 1, 0, st,
                                 nullptr, cfg);
}

void bs_unload(BsCache& cache) {
    for (int i = 0; i < BsCache::kMax; ++i)
        if (cache.mod[i]) {
            hipModuleUnload(cache.mod[i]);
            cache.mod[i] = nullptr;
            cache.fn[i] = nullptr;
        }
}

}  // namespace qf
