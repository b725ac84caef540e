// qf_api.hip -- C ABI of libqf_fec.so (see include/qf_fec.h).
//
// Host-side orchestration only: argument validation, split-table
// construction, workspace management and kernel launches.  All payload
// arithmetic runs in the kernels of qf_kernels.hip; there is no CPU compute
// path for encode or decode.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "gf256_tables.h"
#include "qf_fec.h"
#include "qf_kernels.h"
#include "qf_bs.h"
#include "qf_internal.h"

namespace qf {
const Gf256& gf() {
    static Gf256 g;
    return g;
}
}  // namespace qf

using qf::gf;

namespace qf {
namespace {
thread_local char t_last_error[256];
thread_local char t_refused[96];
}  // namespace

int device_fail(const char* file, int line, hipError_t e) {
    const char* base = strrchr(file, '/');
    base = base ? base + 1 : file;
    // a refused generated-kernel launch returns hipErrorInvalidValue: only
    // then is the refusal noted by note_launch_refused the cause (a refusal a
    // caller recovered from, e.g. by another kernel, is never attached to a
    // later, unrelated failure)
    const bool refused = e == hipErrorInvalidValue && t_refused[0];
    snprintf(t_last_error, sizeof t_last_error, "%s:%d: %s%s%s%s", base, line, hipGetErrorName(e),
             refused ? " (" : "", refused ? t_refused : "", refused ? ")" : "");
    t_refused[0] = 0;
    return QF_EDEVICE;
}

void note_launch_refused(const char* what, int line) {
    snprintf(t_refused, sizeof t_refused, "%s:%d launch refused", what, line);
}

const char* last_error_text() { return t_last_error; }
}  // namespace qf


static inline uint64_t round_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

struct EncTab {
    uint32_t* dev = nullptr;
    uint32_t k_pad = 0;
    uint32_t R = 0;
};

struct qf_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    int num_cus = 256;
    uint32_t* d_tab256 = nullptr;  // 256 split-table records (8 dwords each)
    uint8_t* d_explog = nullptr;   // exp[512] | log[256]
    uint32_t* d_cmbidx = nullptr;  // qf_combine_bs plane-index table (256 x 16 dwords)
    // Cauchy split tables, keyed by (k, r, pass, k_pad)
    std::map<std::tuple<uint32_t, uint32_t, uint32_t, uint32_t>, EncTab> cauchy;
    // custom coefficient tables: pinned host staging + device buffer
    uint32_t* h_custom = nullptr;
    uint32_t* d_custom = nullptr;
    size_t custom_words = 0;
    hipEvent_t custom_done = nullptr;
    // device copies of Cauchy matrices (r x k) for the small-batch encode
    std::map<std::pair<uint32_t, uint32_t>, uint8_t*> small_coef;
    // qf_ctx_set_payload_wait: event the next decode's payload pass waits for
    hipEvent_t payload_wait = nullptr;
    // qf_ctx_set_payload_stream: the stream the next decode's payload pass
    // runs on (has_payload_stream), the acceptance pass's completion event,
    // and whether the decode path launched its payload there itself
    hipStream_t payload_stream = nullptr;
    bool has_payload_stream = false;
    bool payload_on_stream = false;
    hipEvent_t ev_accept = nullptr;
    // recorded after a payload pass on the caller's stream; the context's
    // stream waits for it, so later context work (the next acceptance pass
    // rewriting d_work, qf_sync, workspace growth, destroy) is ordered after
    // that pass's reads of d_work / d_zero
    hipEvent_t ev_payload = nullptr;
    // heterogeneous batch API (qf_*_batch_desc): the generation offset tables
    // of the class being launched (nullptr: strided generations) and the
    // device / pinned buffers holding a call's per-generation metadata
    const uint64_t* offs_in = nullptr;
    bool offs_in_al16 = false;  // every generation's input rows (base + offset) start 16-byte aligned
    const uint64_t* offs_out = nullptr;
    uint8_t* d_desc = nullptr;
    size_t desc_bytes = 0;
    uint8_t* h_desc = nullptr;
    size_t h_desc_bytes = 0;
    hipEvent_t desc_done = nullptr;
    // send batches: one event per download chunk
    std::vector<hipEvent_t> send_ev;
    qf::SendProfile send_prof;
    // receive batches: pinned / device staging (rows, row indices, decode outputs)
    uint8_t* h_recv = nullptr;
    uint8_t* d_recv = nullptr;
    size_t recv_bytes = 0;
    hipEvent_t recv_done = nullptr;
    // decode workspace
    uint8_t* d_work = nullptr;
    size_t work_bytes = 0;
    uint8_t* d_logrows = nullptr;   // GF(2^16) inputs in log form (ctx_gf16_logrows)
    size_t logrows_bytes = 0;
    // zero row read by the syndrome kernel for rows a generation lacks
    uint8_t* d_zero = nullptr;
    size_t zero_bytes = 0;
    // decode pipelining: auxiliary stream + dependency events
    hipStream_t aux = nullptr;
    std::vector<hipEvent_t> dep;
    // host-memory pipeline
    static const int kPipe = 3;
    hipStream_t pstream[kPipe] = {nullptr, nullptr, nullptr};
    uint8_t* d_stage_src[kPipe] = {nullptr, nullptr, nullptr};
    uint8_t* d_stage_rep[kPipe] = {nullptr, nullptr, nullptr};
    size_t stage_src_bytes = 0, stage_rep_bytes = 0;
    // host-memory decode pipeline: one staging block per pipe slot and the
    // slot's events (indices landed, rows landed, decode done)
    uint8_t* d_dstage[kPipe] = {nullptr, nullptr, nullptr};
    size_t dstage_bytes = 0;
    hipEvent_t ev_idx[kPipe] = {nullptr, nullptr, nullptr};
    hipEvent_t ev_rows[kPipe] = {nullptr, nullptr, nullptr};
    hipEvent_t ev_done[kPipe] = {nullptr, nullptr, nullptr};
    // bit-sliced Cauchy kernels (loaded on first use)
    qf::BsCache bs;
    // GF(2^16) log / exp tables (qf_gf16.hip, built on first use)
    uint16_t* d_gf16_log = nullptr;
    uint16_t* d_gf16_exp = nullptr;
    // kernel timing (qf_ctx_profile)
    struct ProfPending {
        size_t slot;
        hipEvent_t a, b;
    };
    struct ProfTotal {
        std::string name;
        uint32_t launches;
        double ms;
    };
    bool prof = false;
    std::vector<ProfPending> prof_pending;
    std::vector<ProfTotal> prof_tot;
    std::vector<hipEvent_t> ev_free;
    std::mutex mu;
    // kernel-path options (QF_OPT_*, qf_ctx_set_option)
    int64_t opt[QF_OPT_COUNT] = {};
};

namespace {

// QF_OPT_* defaults, ranges and the environment variable read once when a
// context is created (include/qf_fec.h).  env_zero: the variable names the
// "off" switch (a non-zero value sets the option to 0).
struct OptDef {
    const char* env;
    int64_t dflt, lo, hi;
    bool env_zero;
};
const OptDef kOpts[QF_OPT_COUNT] = {
    /* FFT_KERNELS */ {"QF_FFT_KERNELS", 1, 0, 1, false},
    /* BITSLICED */ {"QF_DISABLE_BS", 1, 0, 1, true},
    /* ENCODE_SMALL */ {"QF_ENCODE_SMALL", -1, -1, 1, false},
    /* ENCODE_KSPLIT */ {"QF_ENCODE_KSPLIT", 1, 0, 1, false},
    /* ENCODE_V */ {"QF_ENCODE_V", 1, 1, 2, false},
    /* ENCODE_PD */ {"QF_ENCODE_PD", 2, 1, 3, false},
    /* DECODE_PATH */ {nullptr, 0, 0, 2, false},   // QF_DECODE_SYN / QF_DECODE_LEGACY, below
    /* DECODE_KSPLIT */ {"QF_DECODE_KSPLIT", 1, 0, 1, false},
    /* DECODE_SYNW */ {"QF_DECODE_NO_SYNW", 1, 0, 1, true},
    /* DECODE_PD */ {"QF_DECODE_PD", 1, 1, 3, false},
    /* DECODE_CHUNK */ {"QF_DECODE_CHUNK", 0, 0, 1ll << 31, false},
    /* DECODE_OVERLAP */ {"QF_DECODE_OVERLAP", 1, 0, 1, false},
    /* COMBINE_BS */ {"QF_COMBINE_BS", 1, 0, 1, false},
    /* COMBINE_BS_MIN_Q */ {"QF_COMBINE_BS_MIN_Q", 64, 1, 1 << 20, false},
    /* COMBINE_SPLIT */ {"QF_COMBINE_SPLIT", 1, 0, 1, false},
    /* PREPARE_GRID */ {"QF_PREPARE_GRID", 0, 0, 1 << 20, false},
    /* ENC_BLOCKS_PER_CU */ {"QF_ENC_BLOCKS_PER_CU", 0, 0, 64, false},
    /* DEC_BLOCKS_PER_CU */ {"QF_DEC_BLOCKS_PER_CU", 0, 0, 64, false},
    /* SEND_FUSED */ {"QF_SEND_FUSED", 1, 0, 1, false},
    /* SEND_WINDOWS_MIN_TILES */ {"QF_SEND_WINDOWS_MIN_TILES", 256, 0, 1ll << 30, false},
    /* SEND_CHUNKS */ {"QF_SEND_CHUNKS", 1, 1, 8, false},
    /* SEND_PROFILE */ {"QF_SEND_PROFILE", 0, 0, 1, false},
    /* COPY_THREADS */ {"QF_COPY_THREADS", -1, -1, 64, false},
    /* GF16_DYN */ {"QF_GF16_DYN", 1, 0, 1, false},
    /* GF16_LOGIFY */ {"QF_GF16_LOGIFY", 1, 0, 1, false},
    /* GF16_LOGIFY_MIN_BLOCKS */ {"QF_GF16_LOGIFY_MIN_BLOCKS", 4, 0, 1 << 20, false},
    /* GF16_LDS_GJ */ {"QF_GF16_LDS_GJ", 0, 0, 1, false},
    /* GF16_BITSLICED */ {"QF_GF16_BITSLICED", 1, 0, 1, false},
    /* GF16_FFT */ {"QF_GF16_FFT", 1, 0, 2, false},
    /* WIEDEMANN_PROJ */ {"QF_WIEDEMANN_PROJ", 1, 0, 1, false},
    /* GF16_FFT_BS */ {"QF_GF16_FFT_BS", 1, 0, 3, false},
    /* PREPARE_LANES */ {"QF_PREPARE_LANES", 1, 0, 1, false},
    /* ENCODE_MERGED */ {"QF_ENCODE_MERGED", 1, 0, 1, false},
    /* SYNW_SHARED */ {"QF_SYNW_SHARED", 1, 0, 1, false},
    /* COMBINE_WIDE */ {"QF_COMBINE_WIDE", 1, 0, 1, false},
    /* COMBINE_XCD */ {"QF_COMBINE_XCD", 0, 0, 1, false},
    /* COMBINE_JUMP */ {"QF_COMBINE_JUMP", 1, 0, 1, false},
    /* COMBINE_PM24 */ {"QF_COMBINE_PM24", 1, 0, 1, false},
    /* SLIDING_KERNELS */ {"QF_SLIDING_KERNELS", 1, 0, 1, false},
};

int64_t clamp_opt(int o, int64_t v) { return std::min(kOpts[o].hi, std::max(kOpts[o].lo, v)); }

// Defaults, then the environment once (qf_ctx_create only).
void init_opts(qf_ctx* c) {
    for (int o = 0; o < QF_OPT_COUNT; ++o) {
        c->opt[o] = kOpts[o].dflt;
        const char* e = kOpts[o].env ? getenv(kOpts[o].env) : nullptr;
        if (!e || !*e) continue;
        const int64_t v = atoll(e);
        c->opt[o] = kOpts[o].env_zero ? (v ? 0 : 1) : clamp_opt(o, v);
    }
    const char* syn = getenv("QF_DECODE_SYN");
    const char* leg = getenv("QF_DECODE_LEGACY");
    if (leg && atoi(leg)) c->opt[QF_OPT_DECODE_PATH] = 2;
    if (syn && atoi(syn)) c->opt[QF_OPT_DECODE_PATH] = 1;
    c->bs.opt = c->opt;
}

int ensure_device(qf_ctx* ctx) {
    int cur = -1;
    QF_CHECK_HIP(hipGetDevice(&cur));
    if (cur != ctx->device) QF_CHECK_HIP(hipSetDevice(ctx->device));
    return QF_OK;
}

// r x k coefficient matrix (row-major) of the reference's Cauchy
// construction, decoder.rs:280-298.
int cauchy_matrix(uint32_t k, uint32_t r, std::vector<uint8_t>& out) {
    out.assign((size_t)k * r, 0);
    const auto& f = gf();
    for (uint32_t j = 0; j < r; ++j) {
        const uint8_t y = (uint8_t)(k + j);
        for (uint32_t i = 0; i < k; ++i) {
            uint8_t c;
            if (!f.inv((uint8_t)((uint8_t)i ^ y), &c)) return QF_ERANGE;
            out[(size_t)j * k + i] = c;
        }
    }
    return QF_OK;
}

// Split tables for repairs [j0, j0 + ra) of a coefficient matrix: records
// (i, jj) at (i*R + jj)*8 for i < k_pad, zero for i >= k or jj >= ra.
void build_tabs(const uint8_t* coeff_rxk, uint32_t k, uint32_t j0, uint32_t ra, uint32_t R,
                uint32_t k_pad, std::vector<uint32_t>& out) {
    out.assign((size_t)k_pad * R * 8, 0);
    for (uint32_t i = 0; i < k; ++i)
        for (uint32_t jj = 0; jj < ra; ++jj)
            qf::perm_record(coeff_rxk[(size_t)(j0 + jj) * k + i], &out[((size_t)i * R + jj) * 8]);
}

uint32_t pick_R(uint32_t ra) {
    if (ra <= 1) return 1;
    if (ra <= 2) return 2;
    if (ra <= 4) return 4;
    if (ra <= 8) return 8;
    return 16;
}

// Units (16 B) per lane in the encode kernel (QF_OPT_ENCODE_V).
int pick_V(qf_ctx* ctx) { return ctx->opt[QF_OPT_ENCODE_V] == 2 ? 2 : 1; }

// Prefetch depth (row pairs in flight per wave) of the combine kernels.
int pick_PD(qf_ctx* ctx, int opt, int V) {
    int pd = (int)ctx->opt[opt];
    const int maxpd = V == 2 ? 2 : 3;
    if (pd < 1) pd = 1;
    if (pd > maxpd) pd = maxpd;
    return pd;
}

int grow_work(qf_ctx* ctx, size_t bytes) {
    if (bytes <= ctx->work_bytes) return QF_OK;
    if (ctx->d_work) {
        QF_CHECK_HIP(hipStreamSynchronize(ctx->stream));
        QF_CHECK_HIP(hipFree(ctx->d_work));
        ctx->d_work = nullptr;
        ctx->work_bytes = 0;
    }
    const size_t b = round_up(bytes, 1 << 20);
    if (hipMalloc(&ctx->d_work, b) != hipSuccess) return QF_ENOMEM;
    ctx->work_bytes = b;
    return QF_OK;
}

// --- kernel timing ---------------------------------------------------------
hipEvent_t prof_begin(qf_ctx* ctx, hipStream_t st) {
    if (!ctx->prof) return nullptr;
    hipEvent_t a = nullptr;
    if (!ctx->ev_free.empty()) {
        a = ctx->ev_free.back();
        ctx->ev_free.pop_back();
    } else if (hipEventCreate(&a) != hipSuccess) {
        return nullptr;
    }
    if (hipEventRecord(a, st) != hipSuccess) {
        ctx->ev_free.push_back(a);
        return nullptr;
    }
    return a;
}

void prof_end(qf_ctx* ctx, hipStream_t st, hipEvent_t a, const std::string& name) {
    if (!a) return;
    hipEvent_t b = nullptr;
    if (!ctx->ev_free.empty()) {
        b = ctx->ev_free.back();
        ctx->ev_free.pop_back();
    } else if (hipEventCreate(&b) != hipSuccess) {
        ctx->ev_free.push_back(a);
        return;
    }
    hipEventRecord(b, st);
    size_t slot = 0;
    while (slot < ctx->prof_tot.size() && ctx->prof_tot[slot].name != name) ++slot;
    if (slot == ctx->prof_tot.size()) ctx->prof_tot.push_back({name, 0u, 0.0});
    ctx->prof_pending.push_back({slot, a, b});
}

int prof_drain(qf_ctx* ctx) {
    for (auto& p : ctx->prof_pending) {
        QF_CHECK_HIP(hipEventSynchronize(p.b));
        float ms = 0.f;
        QF_CHECK_HIP(hipEventElapsedTime(&ms, p.a, p.b));
        ctx->prof_tot[p.slot].launches++;
        ctx->prof_tot[p.slot].ms += ms;
        ctx->ev_free.push_back(p.a);
        ctx->ev_free.push_back(p.b);
    }
    ctx->prof_pending.clear();
    return QF_OK;
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// device copy of the Cauchy matrix (r x k), cached per (k, r)
int small_coef_matrix(qf_ctx* ctx, uint32_t k, uint32_t r, const uint8_t** out) {
    const auto key = std::make_pair(k, r);
    auto it = ctx->small_coef.find(key);
    if (it == ctx->small_coef.end()) {
        std::vector<uint8_t> cm;
        int s = cauchy_matrix(k, r, cm);
        if (s != QF_OK) return s;
        uint8_t* d = nullptr;
        if (hipMalloc(&d, cm.size()) != hipSuccess) return QF_ENOMEM;
        QF_CHECK_HIP(hipMemcpy(d, cm.data(), cm.size(), hipMemcpyHostToDevice));
        it = ctx->small_coef.emplace(key, d).first;
    }
    *out = it->second;
    return QF_OK;
}

int encode_impl(qf_ctx* ctx, const qf_encode_shape* sh, uint32_t G, const uint8_t* src,
                uint8_t* rep, const uint8_t* coeff, hipStream_t st) {
    const uint32_t k = sh->k, r = sh->r, L = sh->L;
    if (k == 0 || k > 256 || (sh->flags & ~QF_ENCODE_ZERO_TAIL)) return QF_EINVAL;
    if (G == 0 || r == 0 || L == 0) return QF_OK;
    if (!src || !rep) return QF_EINVAL;
    if (!aligned16(src) || !aligned16(rep) || (sh->src_row_stride & 15) || (sh->src_gen_stride & 15) ||
        (sh->rep_row_stride & 15) || (sh->rep_gen_stride & 15))
        return QF_EINVAL;
    if (sh->src_row_stride < L && k > 1) return QF_EINVAL;
    if (sh->rep_row_stride < L && r > 1) return QF_EINVAL;
    const uint32_t Lu = (L + 15) / 16;
    const int V = (r >= 9) ? 1 : pick_V(ctx);  // R = 16 tiles run V = 1 (see launcher)
    const int PD = pick_PD(ctx, QF_OPT_ENCODE_PD, V);
    const uint32_t k_pad = (uint32_t)round_up(k, 2 * (PD + 1));
    const uint32_t passes = (r + 15) / 16;
    std::vector<uint8_t> cm;
    if (!coeff) {
        int s = cauchy_matrix(k, r, cm);
        if (s != QF_OK) return s;
    }
    // Few windows (the per-packet send path): the bit-sliced kernels would
    // run fewer than 64 waves, each doing all k rows x r repairs; the
    // small-batch kernel spreads (generation, repair, unit) over lanes.
    // QF_ENCODE_SMALL=0/1 forces it off/on (tests run both).
    {
        const int force = (int)ctx->opt[QF_OPT_ENCODE_SMALL];
        const bool few = (uint64_t)G * qf::bs_padded_units(L) < 64ull * 128;
        if (!coeff && force != 0 && (force == 1 || few)) {
            const uint8_t* dcoef = nullptr;
            int s = small_coef_matrix(ctx, k, r, &dcoef);
            if (s != QF_OK) return s;
            qf::EncodeSmallArgs a{};
            a.rot = 0;
            a.src_offs = ctx->offs_in;
            a.rep_offs = ctx->offs_out;
            a.src = src;
            a.src_gen_stride = sh->src_gen_stride;
            a.src_row_stride = sh->src_row_stride;
            a.rep = rep;
            a.rep_gen_stride = sh->rep_gen_stride;
            a.rep_row_stride = sh->rep_row_stride;
            a.coef = dcoef;
            a.tab256 = ctx->d_tab256;
            a.k = k;
            a.r = r;
            a.L = L;
            a.Lu = Lu;
            a.G = G;
            hipEvent_t ev = prof_begin(ctx, st);
            QF_CHECK_HIP(qf::launch_encode_small(a, ctx->num_cus, st));
            prof_end(ctx, st, ev, "k_encode_small");
            return QF_OK;
        }
    }
    // Fast path: bit-sliced kernel specialised to the reference's Cauchy
    // matrix of (k, r) (bs_codegen.py), for whole 16-byte rows.
    // (L % 16 != 0: only with the zero tail, whose lane space masks the last unit)
    const bool zero_tail = (sh->flags & QF_ENCODE_ZERO_TAIL) &&
                           (ctx->offs_out ? (r == 1 || sh->rep_row_stride >= 16ull * qf::bs_padded_units(L))
                                          : qf::bs_zero_tail_fits(r, L, sh->rep_row_stride, sh->rep_gen_stride)) &&
                           (uint64_t)G * qf::bs_padded_units(L) < (1ull << 31);
    if (!coeff && ctx->opt[QF_OPT_BITSLICED] && qf::bs_available(k, r) && (L % 16 == 0 || zero_tail) && L >= 32 &&
        sh->src_gen_stride < (1ull << 32) && sh->rep_gen_stride < (1ull << 32) &&
        sh->src_row_stride < (1ull << 32) && sh->rep_row_stride < (1ull << 32) &&
        (uint64_t)G * ((L + 15) / 16) < (1ull << 31)) {
        hipEvent_t ev = prof_begin(ctx, st);
        const char* kname = nullptr;
        QF_CHECK_HIP(qf::bs_launch(ctx->bs, ctx->num_cus, st, k, r, src, rep, sh->src_gen_stride,
                                   sh->rep_gen_stride, sh->src_row_stride, sh->rep_row_stride, L, G,
                                   zero_tail, ctx->offs_in, ctx->offs_out, &kname));
        prof_end(ctx, st, ev, kname ? kname : qf::bs_name(k, r));
        return QF_OK;
    }
    for (uint32_t p = 0; p < passes; ++p) {
        const uint32_t j0 = p * 16;
        const uint32_t ra = std::min<uint32_t>(16, r - j0);
        const uint32_t R = pick_R(ra);
        if ((size_t)k_pad * R * 32 > 160 * 1024) return QF_EINVAL;
        const uint32_t* d_tabs = nullptr;
        if (!coeff) {
            auto key = std::make_tuple(k, r, p, k_pad);
            auto it = ctx->cauchy.find(key);
            if (it == ctx->cauchy.end()) {
                std::vector<uint32_t> h;
                build_tabs(cm.data(), k, j0, ra, R, k_pad, h);
                EncTab t;
                t.k_pad = k_pad;
                t.R = R;
                if (hipMalloc(&t.dev, h.size() * 4) != hipSuccess) return QF_ENOMEM;
                QF_CHECK_HIP(hipMemcpy(t.dev, h.data(), h.size() * 4, hipMemcpyHostToDevice));
                it = ctx->cauchy.emplace(key, t).first;
            }
            d_tabs = it->second.dev;
        } else {
            std::vector<uint32_t> h;
            build_tabs(coeff, k, j0, ra, R, k_pad, h);
            if (h.size() > ctx->custom_words) {
                QF_CHECK_HIP(hipStreamSynchronize(st));
                if (ctx->h_custom) hipHostFree(ctx->h_custom);
                if (ctx->d_custom) hipFree(ctx->d_custom);
                ctx->h_custom = nullptr;
                ctx->d_custom = nullptr;
                const size_t w = round_up(h.size(), 4096);
                if (hipHostMalloc(reinterpret_cast<void**>(&ctx->h_custom), w * 4) != hipSuccess) return QF_ENOMEM;
                if (hipMalloc(&ctx->d_custom, w * 4) != hipSuccess) return QF_ENOMEM;
                ctx->custom_words = w;
            } else {
                // the previous upload / kernel may still read the staging
                QF_CHECK_HIP(hipEventSynchronize(ctx->custom_done));
            }
            memcpy(ctx->h_custom, h.data(), h.size() * 4);
            QF_CHECK_HIP(hipMemcpyAsync(ctx->d_custom, ctx->h_custom, h.size() * 4,
                                        hipMemcpyHostToDevice, st));
            d_tabs = ctx->d_custom;
        }
        qf::CombineUniformArgs a{};
        a.src_offs = ctx->offs_in;
        a.dst_offs = ctx->offs_out;
        a.src = src;
        a.src_gen_stride = sh->src_gen_stride;
        a.src_row_stride = sh->src_row_stride;
        a.dst = rep + (uint64_t)j0 * sh->rep_row_stride;
        a.dst_gen_stride = sh->rep_gen_stride;
        a.dst_row_stride = sh->rep_row_stride;
        a.tabs = d_tabs;
        a.k = k;
        a.k_pad = k_pad;
        a.r_active = ra;
        a.L = L;
        a.Lu = Lu;
        a.total_units = (uint64_t)G * Lu;
        hipEvent_t ev = prof_begin(ctx, st);
        QF_CHECK_HIP(qf::launch_combine_uniform(a, (int)R, V, PD, ctx->num_cus, st));
        prof_end(ctx, st, ev,
                 "k_combine_uniform<" + std::to_string(R) + "," + std::to_string(V) + "," + std::to_string(PD) + ">");
        if (coeff) {
            QF_CHECK_HIP(hipEventRecord(ctx->custom_done, st));
            // a second pass rewrites the staging: wait for this pass first
            if (p + 1 < passes) QF_CHECK_HIP(hipEventSynchronize(ctx->custom_done));
        }
    }
    return QF_OK;
}

// Fused decode of the reference's Cauchy code (no row_coeffs), one pass over
// the received rows:
//   k_decode_prepare_cauchy (lu_out)  acceptance, slot map, LU of C[J,E]
//   qf_cauchy_dec_k*_r*               syndromes (bit-sliced), then the LU
//                                     solve in registers, recovered rows out
// Split-phase decode (qf_ctx_set_payload_wait): the acceptance pass needs the
// row indices only, as the reference's add_packet bookkeeping runs at arrival
// (decoder.rs:678-701); the payload pass (try_decode, decoder.rs:720-783)
// waits for the caller's event, e.g. the H2D copy of the rows.
int payload_gate(qf_ctx* ctx, hipStream_t st) {
    if (ctx->payload_wait) QF_CHECK_HIP(hipStreamWaitEvent(st, ctx->payload_wait, 0));
    return QF_OK;
}

// A device buffer of >= L zero bytes (read in place of absent rows).
int ensure_zero(qf_ctx* ctx, uint32_t L) {
    if (ctx->zero_bytes >= L) return QF_OK;
    if (ctx->d_zero) {
        QF_CHECK_HIP(hipStreamSynchronize(ctx->stream));
        hipFree(ctx->d_zero);
        ctx->d_zero = nullptr;
        ctx->zero_bytes = 0;
    }
    const size_t zb = round_up(L, 4096);
    if (hipMalloc(&ctx->d_zero, zb) != hipSuccess) return QF_ENOMEM;
    QF_CHECK_HIP(hipMemset(ctx->d_zero, 0, zb));
    ctx->zero_bytes = zb;
    return QF_OK;
}

int decode_fused(qf_ctx* ctx, const qf_decode_shape* sh, uint32_t G, const uint8_t* rows,
                 const uint16_t* row_index, const uint32_t* n_rows, uint8_t* rec,
                 uint16_t* rec_index, uint32_t* n_rec, int32_t* status) {
    const uint32_t k = sh->k, r = sh->r, L = sh->L;
    const uint32_t ms = qf::syn_map_stride(k, r);
    const uint32_t lu_stride = 272;
    const size_t off_map = round_up((size_t)G * lu_stride, 256);
    int s = grow_work(ctx, off_map + (size_t)G * ms);
    if (s) return s;
    s = ensure_zero(ctx, L);
    if (s) return s;
    uint8_t* w = ctx->d_work;
    hipStream_t st = ctx->stream;
    qf::PrepareCauchyArgs pa{};
    pa.row_index = row_index;
    pa.n_rows = n_rows;
    pa.explog = ctx->d_explog;
    pa.smap = w + off_map;
    pa.n_out = n_rec;
    pa.rec_index = rec_index;
    pa.status = status;
    pa.k = k;
    pa.r = r;
    pa.e_max = std::min(k, r);
    pa.max_rows = sh->max_rows;
    pa.map_stride = ms;
    pa.G = G;
    pa.lu_out = w;
    pa.lu_stride = lu_stride;
    pa.lanes = ctx->opt[QF_OPT_PREPARE_LANES] != 0 ? 1u : 0u;
    if (ctx->payload_wait) {
        // split phase: the acceptance pass runs beside the caller's other
        // work, on a capped persistent grid (QF_PREPARE_GRID blocks, default
        // one per CU: beside the C2 encode it then takes ~0.42 ms, under the
        // encode, and slows it by ~4 %; the step gains ~2 % (DESIGN 3.2,
        // profiles/r03q_split.jsonl, r03r_split.jsonl); one per two CUs 0.74 ms, 64 blocks
        // 1.39 ms (longer than the encode), 4 per CU slowed the encode 10 %)
        const int64_t pg = ctx->opt[QF_OPT_PREPARE_GRID];
        pa.grid_cap = pg ? (uint32_t)pg : std::max<uint32_t>(1, (uint32_t)ctx->num_cus);
    }
    hipEvent_t ev = prof_begin(ctx, st);
    QF_CHECK_HIP(qf::launch_decode_prepare_cauchy(pa, st));
    prof_end(ctx, st, ev, "k_decode_prepare_lu");
    hipStream_t ps = st;
    if (ctx->has_payload_stream) {   // qf_ctx_set_payload_stream: the payload pass on the caller's stream
        if (!ctx->ev_accept) QF_CHECK_HIP(hipEventCreateWithFlags(&ctx->ev_accept, hipEventDisableTiming));
        QF_CHECK_HIP(hipEventRecord(ctx->ev_accept, st));
        ps = ctx->payload_stream;
        QF_CHECK_HIP(hipStreamWaitEvent(ps, ctx->ev_accept, 0));
        ctx->payload_on_stream = true;
    }
    if (int gs = payload_gate(ctx, ps)) return gs;
    ev = prof_begin(ctx, ps);
    QF_CHECK_HIP(qf::dec_launch(ctx->bs, ctx->num_cus, ps, k, r, rows, rec, sh->rows_gen_stride,
                                sh->rec_gen_stride, sh->row_stride, sh->rec_row_stride, L, G, w + off_map, ms,
                                ctx->d_zero, w, lu_stride, ctx->d_tab256, ctx->offs_in, ctx->offs_out));
    prof_end(ctx, ps, ev, qf::dec_name(&ctx->bs, k, r, L, G, ctx->num_cus));
    if (ps != st) {
        if (!ctx->ev_payload) QF_CHECK_HIP(hipEventCreateWithFlags(&ctx->ev_payload, hipEventDisableTiming));
        QF_CHECK_HIP(hipEventRecord(ctx->ev_payload, ps));
        QF_CHECK_HIP(hipStreamWaitEvent(st, ctx->ev_payload, 0));
    }
    return QF_OK;
}

// Decode payload pass x_E = D s over one pass's coefficient records: the
// bit-sliced qf_combine_bs (wave-uniform coefficients, one generation per
// item) for rows of at least QF_COMBINE_BS_MIN_Q (default 64) lane-chunks of
// 32 bytes, else k_combine_slots; QF_COMBINE_BS=0 keeps k_combine_slots.  The
// bit-sliced kernel reads whole 16-byte units, so with L % 16 != 0 its rows
// must start 16-byte aligned (strided, aligned base and strides).
static bool combine_bs_ok(qf_ctx* ctx, const qf::CombineSlotsArgs& a, bool offs_al16) {
    if (!ctx->opt[QF_OPT_COMBINE_BS] || !qf::cmb_available()) return false;
    const uint32_t min_q = (uint32_t)ctx->opt[QF_OPT_COMBINE_BS_MIN_Q];
    // (Lu >= 2: the partial last unit is then always some lane's unit B)
    if (a.Lu < 2 || (a.Lu + 1) / 2 < min_q) return false;
    // (32-bit strides in the kernel: row j of the 16 outputs at j * dst stride)
    if (a.row_stride >= (1ull << 32) || 16ull * a.dst_row_stride >= (1ull << 32) || a.coef_gen_stride >= (1ull << 32))
        return false;
    if (a.L % 16 && ((a.rows_offs && !offs_al16) ||
                     ((uintptr_t)a.rows | a.row_stride | (a.rows_offs ? 0 : a.rows_gen_stride)) % 16))
        return false;
    return true;
}

static hipError_t combine_payload(qf_ctx* ctx, const qf::CombineSlotsArgs& a, int PD, hipStream_t st,
                                  std::string* name) {
    // (rows_offs is the context's input table on the general path only)
    if (combine_bs_ok(ctx, a, a.rows_offs == ctx->offs_in && ctx->offs_in_al16)) {
        if (name) *name = qf::cmb_kernel_name(ctx->bs, a);
        return qf::cmb_launch(ctx->bs, ctx->num_cus, st, a, ctx->d_cmbidx);
    }
    const bool split_ok = ctx->opt[QF_OPT_COMBINE_SPLIT] != 0;
    if (name) {
        const bool split = split_ok && (a.total_units + 63) / 64 <= (uint64_t)ctx->num_cus;
        *name = split ? std::string("k_combine_slots_split") : "k_combine_slots<" + std::to_string(PD) + ">";
    }
    return qf::launch_combine_slots(a, PD, ctx->num_cus, st, split_ok);
}


// Decode of Cauchy codes with more repairs than a syndrome kernel holds
// (r <= 64, e <= 64) when the encode kernels of (k, r) exist:
//   k_decode_prepare_cauchy  acceptance, slot map, D = C[J,E]^-1 (closed form)
//   k_gather_sources         x' = accepted sources in order, erased ones zero
//   qf_cauchy_bs_k*_r*       C x' = C[., S] x_S                (bit-sliced)
//   k_xor_repairs            s_J = p_J ^ C[J, S] x_S
//   k_combine_slots          x_E = D s_J, passes of 16 outputs
int decode_cauchy_enc(qf_ctx* ctx, const qf_decode_shape* sh, uint32_t G, const uint8_t* rows,
                      const uint16_t* row_index, const uint32_t* n_rows, uint8_t* rec,
                      uint16_t* rec_index, uint32_t* n_rec, int32_t* status) {
    const uint32_t k = sh->k, r = sh->r, L = sh->L;
    const uint32_t e_max = std::min(k, r), passes = (e_max + 15) / 16;
    const uint32_t ms = (uint32_t)round_up(k + r, 16);
    const uint64_t cgs = (uint64_t)(r + 1) * 16;
    const uint64_t Lp = 16ull * qf::bs_padded_units(L);  // zero-tail encode rows
    const uint32_t Lu = (L + 15) / 16;
    // long rows (padded units >= 128): the syndrome passes read the received
    // rows through the slot map themselves (qf_cauchy_synw_*), no gather
    const bool synw = qf::synw_available(k, r) && Lp >= 16 * 128 && ctx->opt[QF_OPT_DECODE_SYNW];
    // generations per chunk: gathered sources + syndromes of about 1 GiB
    const uint64_t chunk = std::max<uint64_t>(
        1, std::min<uint64_t>(G, (1ull << 30) / ((uint64_t)((synw ? 0 : k) + r) * Lp)));
    const size_t off_bound = round_up((size_t)passes * G * cgs, 256);
    const size_t off_map = round_up(off_bound + (size_t)G * 4, 256);
    const size_t off_x = round_up(off_map + (size_t)G * ms, 256);
    const size_t off_syn = round_up(off_x + (synw ? 0 : (size_t)chunk * k * Lp), 256);
    int s = grow_work(ctx, off_syn + (size_t)chunk * r * Lp);
    if (s) return s;
    if (synw && (s = ensure_zero(ctx, (uint32_t)Lp)) != QF_OK) return s;
    uint8_t* w = ctx->d_work;
    uint32_t* d_bound = reinterpret_cast<uint32_t*>(w + off_bound);
    hipStream_t st = ctx->stream;
    qf::PrepareCauchyArgs pa{};
    pa.row_index = row_index;
    pa.n_rows = n_rows;
    pa.explog = ctx->d_explog;
    pa.coef_out = w;
    pa.smap = w + off_map;
    pa.n_out = n_rec;
    pa.bound = d_bound;
    pa.rec_index = rec_index;
    pa.status = status;
    pa.k = k;
    pa.r = r;
    pa.e_max = e_max;
    pa.max_rows = sh->max_rows;
    pa.map_stride = ms;
    pa.G = G;
    hipEvent_t ev = prof_begin(ctx, st);
    QF_CHECK_HIP(qf::launch_decode_prepare_cauchy(pa, st));
    prof_end(ctx, st, ev, "k_decode_prepare_cauchy");
    if (int gs = payload_gate(ctx, st)) return gs;
    const int PD = pick_PD(ctx, QF_OPT_DECODE_PD, 1);
    for (uint64_t g0 = 0; g0 < G; g0 += chunk) {
        const uint32_t Gc = (uint32_t)std::min<uint64_t>(chunk, G - g0);
        if (synw) {
            ev = prof_begin(ctx, st);
            QF_CHECK_HIP(qf::synw_launch(ctx->bs, ctx->num_cus, st, k, r,
                                         ctx->offs_in ? rows : rows + g0 * sh->rows_gen_stride, w + off_syn,
                                         ctx->offs_in ? 0 : sh->rows_gen_stride, (uint64_t)r * Lp, sh->row_stride, Lp, L,
                                         Gc, w + off_map + g0 * ms, ms, ctx->d_zero, d_bound + g0,
                                         ctx->offs_in ? ctx->offs_in + g0 : nullptr));
            prof_end(ctx, st, ev, std::string("qf_cauchy_synw_k") + std::to_string(k) + "_r" + std::to_string(r));
        }
        qf::GatherArgs ga{};
        ga.rows = rows + g0 * sh->rows_gen_stride;
        ga.rows_gen_stride = sh->rows_gen_stride;
        ga.rows_offs = ctx->offs_in ? ctx->offs_in + g0 : nullptr;
        ga.row_stride = sh->row_stride;
        ga.smap = w + off_map + g0 * ms;
        ga.map_stride = ms;
        ga.out = w + off_x;
        ga.out_gen_stride = (uint64_t)k * Lp;
        ga.out_row_stride = Lp;
        ga.k = k;
        ga.r = r;
        ga.Lu = Lu;
        ga.G = Gc;
        if (!synw) {
            ev = prof_begin(ctx, st);
            QF_CHECK_HIP(qf::launch_gather_sources(ga, ctx->num_cus, st));
            prof_end(ctx, st, ev, "k_gather_sources");
            ev = prof_begin(ctx, st);
            const char* kname = nullptr;
            QF_CHECK_HIP(qf::bs_launch(ctx->bs, ctx->num_cus, st, k, r, w + off_x, w + off_syn, (uint64_t)k * Lp,
                                       (uint64_t)r * Lp, Lp, Lp, L, Gc, true, nullptr, nullptr, &kname));
            prof_end(ctx, st, ev, kname ? kname : qf::bs_name(k, r));
            ga.out = w + off_syn;
            ga.out_gen_stride = (uint64_t)r * Lp;
            ev = prof_begin(ctx, st);
            QF_CHECK_HIP(qf::launch_xor_repairs(ga, ctx->num_cus, st));
            prof_end(ctx, st, ev, "k_xor_repairs");
        }
        // every pass in one pass-major launch (QF_ENCODE_MERGED, the
        // bit-sliced payload kernel): one pass's last, partly filled round of
        // workgroups overlaps the next pass's first
        bool pm = false;
        for (uint32_t p = 0; p < passes && !pm; ++p) {
            qf::CombineSlotsArgs a{};
            a.rows = w + off_syn;
            a.rows_gen_stride = (uint64_t)r * Lp;
            a.row_stride = Lp;
            a.dst = rec + g0 * sh->rec_gen_stride + (uint64_t)p * 16 * sh->rec_row_stride;
            a.dst_gen_stride = sh->rec_gen_stride;
            a.dst_offs = ctx->offs_out ? ctx->offs_out + g0 : nullptr;
            a.dst_row_stride = sh->rec_row_stride;
            a.coef = w + ((uint64_t)p * G + g0) * cgs;
            a.coef_gen_stride = cgs;
            a.n_out = n_rec + g0;
            a.bound = d_bound + g0;
            a.tab256 = ctx->d_tab256;
            a.pass = p;
            a.L = L;
            a.Lu = Lu;
            a.zero_slot = r;
            a.total_units = (uint64_t)Gc * Lu;
            ev = prof_begin(ctx, st);
            std::string cname;
            pm = p == 0 && ctx->opt[QF_OPT_ENCODE_MERGED] &&
                 qf::cmb_pass_major_ok(passes, sh->rec_row_stride, (uint64_t)G * cgs) &&
                 combine_bs_ok(ctx, a, a.rows_offs == ctx->offs_in && ctx->offs_in_al16);
            if (pm) {
                cname = qf::cmb_kernel_name(ctx->bs, a, passes, (uint64_t)G * cgs, e_max);
                QF_CHECK_HIP(qf::cmb_launch(ctx->bs, ctx->num_cus, st, a, ctx->d_cmbidx, passes, (uint64_t)G * cgs,
                                            e_max));
            } else {
                QF_CHECK_HIP(combine_payload(ctx, a, PD, st, &cname));
            }
            prof_end(ctx, st, ev, cname);
        }
    }
    return QF_OK;
}

// Decode of the reference's Cauchy code by syndromes (no row_coeffs):
//   k_decode_prepare_cauchy  acceptance, slot map, D = C[J,E]^-1 (closed form)
//   qf_cauchy_syn_k*_r*      s_j = p_j ^ sum_{i present} C[j][i] x_i  (bit-sliced)
//   k_combine_slots          x_E = D s_J
int decode_cauchy(qf_ctx* ctx, const qf_decode_shape* sh, uint32_t G, const uint8_t* rows,
                  const uint16_t* row_index, const uint32_t* n_rows, uint8_t* rec,
                  uint16_t* rec_index, uint32_t* n_rec, int32_t* status) {
    const uint32_t k = sh->k, r = sh->r, L = sh->L;
    const uint32_t ms = qf::syn_map_stride(k, r);
    const uint64_t coef_gen_stride = (uint64_t)(r + 1) * 16;
    // Optional pipelining of stage A (syndromes) and stage B (v_perm combine)
    // over chunks of QF_DECODE_CHUNK generations: B of chunk c on an
    // auxiliary stream while A of chunk c + 1 runs on the context's stream
    // (double-buffered syndromes); QF_DECODE_OVERLAP=0 keeps both on the
    // context's stream.  Measured at C3 (profiles/r01_decode_pipeline.json):
    // the two kernels slow each other down when co-resident (A is not idle on
    // the VALU), so 8 chunks with overlap take 2.49 ms and one chunk 2.25 ms:
    // the default is one chunk.
    uint64_t chunk = G;
    if (ctx->opt[QF_OPT_DECODE_CHUNK] > 0) chunk = std::min<uint64_t>((uint64_t)ctx->opt[QF_OPT_DECODE_CHUNK], G);
    const uint64_t n_chunks = (G + chunk - 1) / chunk;
    const bool overlap = n_chunks > 1 && ctx->opt[QF_OPT_DECODE_OVERLAP] != 0;
    // syndrome rows: the padded lane space of the syndrome kernel (whole
    // 128-B lines per row; qf_bs.h)
    const uint64_t syn_rs = 16ull * qf::bs_padded_units(L);
    const size_t syn_bytes = round_up((size_t)chunk * r * syn_rs, 256);
    const size_t off_bound = round_up((size_t)G * coef_gen_stride, 256);
    const size_t off_map = round_up(off_bound + (size_t)G * 4, 256);
    const size_t off_syn = round_up(off_map + (size_t)G * ms, 256);
    const size_t total = off_syn + syn_bytes * (overlap ? 2 : 1);
    int s = grow_work(ctx, total);
    if (s) return s;
    uint8_t* w = ctx->d_work;
    uint32_t* d_bound = reinterpret_cast<uint32_t*>(w + off_bound);
    s = ensure_zero(ctx, L);
    if (s) return s;
    hipStream_t st = ctx->stream, sb = ctx->stream;
    if (overlap) {
        if (!ctx->aux) QF_CHECK_HIP(hipStreamCreateWithFlags(&ctx->aux, hipStreamNonBlocking));
        sb = ctx->aux;
        while (ctx->dep.size() < 2 * n_chunks + 1) {
            hipEvent_t e;
            QF_CHECK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            ctx->dep.push_back(e);
        }
    }
    qf::PrepareCauchyArgs pa{};
    pa.row_index = row_index;
    pa.n_rows = n_rows;
    pa.explog = ctx->d_explog;
    pa.coef_out = w;
    pa.smap = w + off_map;
    pa.n_out = n_rec;
    pa.bound = d_bound;
    pa.rec_index = rec_index;
    pa.status = status;
    pa.k = k;
    pa.r = r;
    pa.e_max = std::min(k, r);
    pa.max_rows = sh->max_rows;
    pa.map_stride = ms;
    pa.G = G;
    hipEvent_t ev = prof_begin(ctx, st);
    QF_CHECK_HIP(qf::launch_decode_prepare_cauchy(pa, st));
    prof_end(ctx, st, ev, "k_decode_prepare_cauchy");
    if (int gs = payload_gate(ctx, st)) return gs;
    const int PD = pick_PD(ctx, QF_OPT_DECODE_PD, 1);
    for (uint64_t c = 0; c < n_chunks; ++c) {
        const uint64_t g0 = c * chunk;
        const uint32_t Gc = (uint32_t)std::min<uint64_t>(chunk, G - g0);
        uint8_t* syn = w + off_syn + (overlap ? (c & 1) * syn_bytes : 0);
        hipEvent_t evA = overlap ? ctx->dep[2 * c] : nullptr, evB = overlap ? ctx->dep[2 * c + 1] : nullptr;
        if (overlap && c >= 2) QF_CHECK_HIP(hipStreamWaitEvent(st, ctx->dep[2 * (c - 2) + 1], 0));
        ev = prof_begin(ctx, st);
        QF_CHECK_HIP(qf::syn_launch(ctx->bs, ctx->num_cus, st, k, r, rows + g0 * sh->rows_gen_stride, syn,
                                    sh->rows_gen_stride, (uint64_t)r * syn_rs, sh->row_stride, syn_rs, L, Gc,
                                    w + off_map + g0 * ms, ms, ctx->d_zero,
                                    ctx->offs_in ? ctx->offs_in + g0 : nullptr));
        prof_end(ctx, st, ev, qf::syn_name(k, r));
        if (overlap) {
            QF_CHECK_HIP(hipEventRecord(evA, st));
            QF_CHECK_HIP(hipStreamWaitEvent(sb, evA, 0));
        }
        qf::CombineSlotsArgs a{};
        a.rows = syn;
        a.rows_gen_stride = (uint64_t)r * syn_rs;
        a.row_stride = syn_rs;
        a.dst = rec + g0 * sh->rec_gen_stride;
        a.dst_gen_stride = sh->rec_gen_stride;
        a.dst_offs = ctx->offs_out ? ctx->offs_out + g0 : nullptr;
        a.dst_row_stride = sh->rec_row_stride;
        a.coef = w + g0 * coef_gen_stride;
        a.coef_gen_stride = coef_gen_stride;
        a.n_out = n_rec + g0;
        a.bound = d_bound + g0;
        a.tab256 = ctx->d_tab256;
        a.pass = 0;
        a.L = L;
        a.Lu = (L + 15) / 16;
        a.zero_slot = r;
        a.total_units = (uint64_t)Gc * a.Lu;
        ev = prof_begin(ctx, sb);
        std::string cname;
        QF_CHECK_HIP(combine_payload(ctx, a, PD, sb, &cname));
        prof_end(ctx, sb, ev, cname);
        if (overlap) QF_CHECK_HIP(hipEventRecord(evB, sb));
    }
    if (overlap) {
        // the caller's stream sees the whole decode: join the last B launches
        QF_CHECK_HIP(hipStreamWaitEvent(st, ctx->dep[2 * (n_chunks - 1) + 1], 0));
        if (n_chunks >= 2) QF_CHECK_HIP(hipStreamWaitEvent(st, ctx->dep[2 * (n_chunks - 2) + 1], 0));
    }
    return QF_OK;
}

int desc_stage(qf_ctx* ctx, size_t bytes);
int desc_upload(qf_ctx* ctx, size_t bytes);

}  // namespace

namespace qf {
int ctx_lock(qf_ctx* ctx, std::unique_lock<std::mutex>& lk) {
    lk = std::unique_lock<std::mutex>(ctx->mu);
    return ensure_device(ctx);
}
hipStream_t ctx_stream(qf_ctx* ctx) { return ctx->stream; }
int ctx_num_cus(qf_ctx* ctx) { return ctx->num_cus; }
bool small_encode_enabled(qf_ctx* ctx) { return ctx->opt[QF_OPT_ENCODE_SMALL] != 0; }
int64_t ctx_opt(qf_ctx* ctx, int opt) { return (opt >= 0 && opt < QF_OPT_COUNT) ? ctx->opt[opt] : 0; }
int encode_ring_window(qf_ctx* ctx, uint32_t k, uint32_t first, uint32_t count, uint32_t L, const uint8_t* ring,
                       uint64_t stride, uint32_t rot, uint8_t* rep, uint64_t rep_stride, const uint8_t* fresh,
                       uint8_t* fresh_dst, uint32_t fresh_units) {
    if (!ctx || !ring || !rep || k == 0 || count == 0 || rot >= k) return QF_EINVAL;
    if ((uint64_t)k + first + count > 256) return QF_ERANGE;  // gf_inv(0)
    if (L == 0) return QF_OK;
    std::lock_guard<std::mutex> g(ctx->mu);
    int s = ensure_device(ctx);
    if (s) return s;
    const uint8_t* dcoef = nullptr;
    s = small_coef_matrix(ctx, k, first + count, &dcoef);  // Cauchy row j depends on (k, j) only
    if (s != QF_OK) return s;
    qf::EncodeSmallArgs a{};
    a.src = ring;
    a.src_gen_stride = (uint64_t)k * stride;
    a.src_row_stride = stride;
    a.rep = rep;
    a.rep_gen_stride = (uint64_t)count * rep_stride;
    a.rep_row_stride = rep_stride;
    a.coef = dcoef + (size_t)first * k;
    a.tab256 = ctx->d_tab256;
    a.k = k;
    a.r = count;
    a.L = L;
    a.Lu = (L + 15) / 16;
    a.G = 1;
    a.rot = rot;
    hipEvent_t ev = prof_begin(ctx, ctx->stream);
    if (fresh) {
        if (!fresh_dst || rep_stride < 16ull * a.Lu || stride < 16ull * fresh_units ||
            fresh_units > qf::SEND_PKT_UNITS)
            return QF_EINVAL;
        a.fresh_dst = fresh_dst;
        a.fresh_units = fresh_units;
        QF_CHECK_HIP(qf::launch_send_window(a, fresh, 16u * fresh_units, ctx->stream));
        prof_end(ctx, ctx->stream, ev, "k_send_window");
        return QF_OK;
    }
    QF_CHECK_HIP(qf::launch_encode_small(a, ctx->num_cus, ctx->stream));
    prof_end(ctx, ctx->stream, ev, "k_encode_small");
    return QF_OK;
}
int encode_ring_windows(qf_ctx* ctx, uint32_t k, uint32_t r, uint32_t G, uint32_t max_L, const uint8_t* src,
                        uint8_t* rep, const RingWin* wins) {
    if (!ctx || !src || !rep || !wins || k == 0 || r == 0) return QF_EINVAL;
    if ((uint64_t)k + r > 256) return QF_ERANGE;  // gf_inv(0)
    if (G == 0 || max_L == 0) return QF_OK;
    const uint8_t* dcoef = nullptr;
    int s = small_coef_matrix(ctx, k, r, &dcoef);
    if (s != QF_OK) return s;
    qf::EncodeSmallArgs a{};
    a.src = src;
    a.rep = rep;
    a.coef = dcoef;
    a.tab256 = ctx->d_tab256;
    a.k = k;
    a.r = r;
    a.L = max_L;
    a.Lu = (max_L + 15) / 16;
    a.G = G;
    a.wins = wins;
    // all repairs of a tile per block once there are enough tiles to fill
    // the chip; below that the one-repair tiles spread a few windows wider
    const uint64_t min_tiles = (uint64_t)ctx->opt[QF_OPT_SEND_WINDOWS_MIN_TILES];
    const uint64_t tiles = (uint64_t)G * ((a.Lu + 63) / 64);
    const bool wide = tiles >= min_tiles;
    hipEvent_t ev = prof_begin(ctx, ctx->stream);
    QF_CHECK_HIP(wide ? qf::launch_encode_windows(a, ctx->num_cus, ctx->stream)
                      : qf::launch_encode_small(a, ctx->num_cus, ctx->stream));
    prof_end(ctx, ctx->stream, ev, wide ? "k_encode_windows" : "k_encode_small");
    return QF_OK;
}
int ctx_desc_buffers(qf_ctx* ctx, size_t bytes, uint8_t** h, uint8_t** d) {
    int s = desc_stage(ctx, bytes);
    if (s != QF_OK) return s;
    *h = ctx->h_desc;
    *d = ctx->d_desc;
    return QF_OK;
}
int ctx_desc_upload(qf_ctx* ctx, size_t bytes) { return desc_upload(ctx, bytes); }
int ctx_recv_buffers(qf_ctx* ctx, size_t bytes, uint8_t** h, uint8_t** d) {
    if (!ctx->recv_done) QF_CHECK_HIP(hipEventCreateWithFlags(&ctx->recv_done, hipEventDisableTiming));
    else QF_CHECK_HIP(hipEventSynchronize(ctx->recv_done));
    if (bytes > ctx->recv_bytes) {
        QF_CHECK_HIP(hipStreamSynchronize(ctx->stream));
        if (ctx->h_recv) hipHostFree(ctx->h_recv);
        if (ctx->d_recv) hipFree(ctx->d_recv);
        ctx->h_recv = nullptr;
        ctx->d_recv = nullptr;
        ctx->recv_bytes = 0;
        const size_t b = round_up(bytes, 1 << 20);
        if (hipHostMalloc(reinterpret_cast<void**>(&ctx->h_recv), b) != hipSuccess) return QF_ENOMEM;
        if (hipMalloc(&ctx->d_recv, b) != hipSuccess) return QF_ENOMEM;
        ctx->recv_bytes = b;
    }
    *h = ctx->h_recv;
    *d = ctx->d_recv;
    return QF_OK;
}
int ctx_recv_release(qf_ctx* ctx) {
    QF_CHECK_HIP(hipEventRecord(ctx->recv_done, ctx->stream));
    return QF_OK;
}
SendProfile* ctx_send_profile(qf_ctx* ctx) { return &ctx->send_prof; }

int ctx_send_events(qf_ctx* ctx, uint32_t n, hipEvent_t** out) {
    while (ctx->send_ev.size() < n) {
        hipEvent_t e = nullptr;
        QF_CHECK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        ctx->send_ev.push_back(e);
    }
    *out = ctx->send_ev.data();
    return QF_OK;
}
const uint32_t* ctx_tab256(qf_ctx* ctx) { return ctx->d_tab256; }
int ctx_gf16_logrows(qf_ctx* ctx, size_t bytes, uint8_t** out) {
    if (bytes > ctx->logrows_bytes) {
        if (ctx->d_logrows) {
            QF_CHECK_HIP(hipStreamSynchronize(ctx->stream));
            QF_CHECK_HIP(hipFree(ctx->d_logrows));
            ctx->d_logrows = nullptr;
            ctx->logrows_bytes = 0;
        }
        const size_t b = round_up(bytes, 1 << 20);
        if (hipMalloc(&ctx->d_logrows, b) != hipSuccess) return QF_ENOMEM;
        ctx->logrows_bytes = b;
    }
    *out = ctx->d_logrows;
    return QF_OK;
}
int ctx_work(qf_ctx* ctx, size_t bytes, uint8_t** out) {
    int s = grow_work(ctx, bytes);
    if (s) return s;
    *out = ctx->d_work;
    return QF_OK;
}
int ctx_gf16_tables(qf_ctx* ctx, const uint16_t** log, const uint16_t** exp) {
    if (!ctx->d_gf16_log) {
        // log 0: 0xFFFF (no product); entries 65,536.. hold the Zech logs
        // Z[d] = log(1 + alpha^d) (Z[0] = log 0) for ctx_gf16_zech
        std::vector<uint16_t> lg(2 * 65536, 0xFFFF), ex(2 * 65535);
        uint32_t x = 1;
        for (uint32_t i = 0; i < 65535; ++i) {  // generator 2 of GF(2^16) mod 0x1100B
            ex[i] = ex[i + 65535] = (uint16_t)x;
            lg[x] = (uint16_t)i;
            x <<= 1;
            if (x & 0x10000u) x ^= 0x1100Bu;
        }
        for (uint32_t d = 1; d < 65535; ++d) lg[65536 + d] = lg[1u ^ ex[d]];
        uint16_t *dl = nullptr, *de = nullptr;
        if (hipMalloc(&dl, lg.size() * 2) != hipSuccess) return QF_ENOMEM;
        if (hipMalloc(&de, ex.size() * 2) != hipSuccess) {
            hipFree(dl);
            return QF_ENOMEM;
        }
        QF_CHECK_HIP(hipMemcpy(dl, lg.data(), lg.size() * 2, hipMemcpyHostToDevice));
        QF_CHECK_HIP(hipMemcpy(de, ex.data(), ex.size() * 2, hipMemcpyHostToDevice));
        ctx->d_gf16_log = dl;
        ctx->d_gf16_exp = de;
    }
    *log = ctx->d_gf16_log;
    *exp = ctx->d_gf16_exp;
    return QF_OK;
}
int ctx_gf16_zech(qf_ctx* ctx, const uint16_t** zech) {
    const uint16_t *lg, *ex;
    const int s = ctx_gf16_tables(ctx, &lg, &ex);
    if (s) return s;
    *zech = lg + 65536;
    return QF_OK;
}
hipEvent_t ctx_prof_begin(qf_ctx* ctx, hipStream_t st) { return prof_begin(ctx, st); }
void ctx_prof_end(qf_ctx* ctx, hipStream_t st, hipEvent_t ev, const std::string& name) {
    prof_end(ctx, st, ev, name);
}

hipError_t launch_frame_batch(const uint8_t* src, const uint8_t* rep, const qf_encode_shape& sh, uint32_t G,
                              uint8_t* frames, uint64_t frame_stride, uint32_t* frame_len,
                              const uint8_t* explog, int num_cus, hipStream_t st);
hipError_t launch_parse_frames(const uint8_t* frames, uint64_t frame_stride, const uint32_t* frame_len,
                               const uint64_t* ids, const uint32_t* n_frames, uint32_t k, uint32_t r, uint32_t L,
                               uint32_t G, uint32_t max_rows, uint8_t* rows, uint64_t row_stride,
                               uint64_t rows_gen_stride, uint16_t* row_index, uint32_t* n_rows,
                               int32_t* frame_status, const uint8_t* explog, hipStream_t st);
}  // namespace qf

extern "C" {

int qf_abi_version(void) { return QF_ABI_VERSION; }


const char* qf_last_error(void) { return qf::last_error_text(); }

const char* qf_strerror(int s) {
    switch (s) {
        case QF_OK: return "ok";
        case QF_EINVAL: return "invalid argument";
        case QF_ERANGE: return "coefficient undefined (gf_inv(0): k + r > 256)";
        case QF_ENOTREADY: return "not ready (window not full / fewer than k rows)";
        case QF_ERANK: return "decode matrix singular";
        case QF_EDEVICE: return "HIP device error";
        case QF_ENOMEM: return "out of memory";
        case QF_ETOOSMALL: return "buffer too short";
        default: return "unknown status";
    }
}

int qf_gf256_init(void) {
    (void)gf();
    return QF_OK;
}

uint8_t qf_gf256_mul(uint8_t a, uint8_t b) { return gf().mul(a, b); }

uint8_t qf_gf256_mul_add(uint8_t a, uint8_t b, uint8_t c) { return (uint8_t)(gf().mul(a, b) ^ c); }

int qf_gf256_inv(uint8_t a, uint8_t* out) {
    if (!out) return QF_EINVAL;
    return gf().inv(a, out) ? QF_OK : QF_ERANGE;
}

int qf_cauchy_coeffs(uint32_t k, uint32_t r, uint8_t* out_rxk) {
    if (!out_rxk && k && r) return QF_EINVAL;
    std::vector<uint8_t> m;
    int s = cauchy_matrix(k, r, m);
    if (s != QF_OK) return s;
    if (!m.empty()) memcpy(out_rxk, m.data(), m.size());
    return QF_OK;
}

int qf_ctx_create(int device, void* stream, qf_ctx** out) {
    if (!out) return QF_EINVAL;
    *out = nullptr;
    int n = 0;
    QF_CHECK_HIP(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) return qf::device_fail(__FILE__, __LINE__, hipErrorInvalidDevice);
    QF_CHECK_HIP(hipSetDevice(device));
    qf_ctx* c = new qf_ctx();
    c->device = device;
    init_opts(c);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->num_cus = prop.multiProcessorCount;
    if (stream == QF_STREAM_NULL) {
        c->stream = nullptr;   // the null stream (not owned)
    } else if (stream) {
        c->stream = reinterpret_cast<hipStream_t>(stream);
    } else {
        if (hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) {
            delete c;
            return qf::device_fail(__FILE__, __LINE__, e);
        }
        c->own_stream = true;
    }
    // value-indexed split tables and exp/log tables
    std::vector<uint32_t> tab(256 * 8);
    for (int v = 0; v < 256; ++v) qf::perm_record((uint8_t)v, &tab[v * 8]);
    std::vector<uint8_t> el(768);
    memcpy(el.data(), gf().exp, 512);
    memcpy(el.data() + 512, gf().log, 256);
    // plane indices of the bit-sliced payload pass (bs_codegen.cmb_index_table):
    // dword 2p / 2p + 1 of record c = low / high nibble of row p of M_c
    std::vector<uint32_t> cidx(256 * 16);
    for (int v = 0; v < 256; ++v) {
        uint8_t rows[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int a = 0; a < 8; ++a) {
            const uint8_t col = gf().mul((uint8_t)v, (uint8_t)(1u << a));
            for (int b = 0; b < 8; ++b) rows[b] |= (uint8_t)(((col >> b) & 1u) << a);
        }
        for (int p = 0; p < 8; ++p) {
            cidx[v * 16 + 2 * p] = rows[p] & 15u;
            cidx[v * 16 + 2 * p + 1] = rows[p] >> 4;
        }
    }
    bool ok = hipMalloc(&c->d_tab256, tab.size() * 4) == hipSuccess &&
              hipMalloc(&c->d_explog, 768) == hipSuccess &&
              hipMalloc(&c->d_cmbidx, cidx.size() * 4) == hipSuccess &&
              hipMemcpy(c->d_cmbidx, cidx.data(), cidx.size() * 4, hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(c->d_tab256, tab.data(), tab.size() * 4, hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(c->d_explog, el.data(), 768, hipMemcpyHostToDevice) == hipSuccess &&
              hipEventCreateWithFlags(&c->custom_done, hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        const hipError_t e = hipGetLastError();
        qf_ctx_destroy(c);
        return qf::device_fail(__FILE__, __LINE__, e != hipSuccess ? e : hipErrorOutOfMemory);
    }
    *out = c;
    return QF_OK;
}

int qf_ctx_destroy(qf_ctx* c) {
    if (!c) return QF_OK;
    if (const uint64_t n = c->send_prof.calls) {   // QF_OPT_SEND_PROFILE (qf_objects.hip encoders_send_batch)
        const qf::SendProfile& p = c->send_prof;
        fprintf(stderr, "[qf send batch] ctx %p: %llu calls, us/call: stage %.1f  launch %.1f  wait %.1f  copy-out %.1f\n",
                (void*)c, (unsigned long long)n, 1e6 * p.t[0] / n, 1e6 * p.t[1] / n, 1e6 * p.t[2] / n, 1e6 * p.t[3] / n);
        fprintf(stderr, "[qf send batch] ctx %p: stage = host %.1f + buffers %.1f + packets %.1f + upload %.1f\n",
                (void*)c, 1e6 * p.u[0] / n, 1e6 * p.u[1] / n, 1e6 * p.u[2] / n, 1e6 * p.u[3] / n);
    }
    hipSetDevice(c->device);
    // (a null stream is QF_STREAM_NULL's: synchronising it is valid and
    // needed before the buffers below are freed)
    hipStreamSynchronize(c->stream);
    for (auto& kv : c->cauchy) hipFree(kv.second.dev);
    for (auto& kv : c->small_coef) hipFree(kv.second);
    if (c->d_tab256) hipFree(c->d_tab256);
    if (c->d_logrows) hipFree(c->d_logrows);
    if (c->d_explog) hipFree(c->d_explog);
    if (c->d_cmbidx) hipFree(c->d_cmbidx);
    if (c->h_custom) hipHostFree(c->h_custom);
    if (c->d_custom) hipFree(c->d_custom);
    if (c->custom_done) hipEventDestroy(c->custom_done);
    if (c->d_work) hipFree(c->d_work);
    if (c->d_desc) hipFree(c->d_desc);
    if (c->h_desc) hipHostFree(c->h_desc);
    if (c->desc_done) hipEventDestroy(c->desc_done);
    if (c->ev_accept) hipEventDestroy(c->ev_accept);
    if (c->ev_payload) hipEventDestroy(c->ev_payload);
    for (hipEvent_t e : c->send_ev) hipEventDestroy(e);
    if (c->recv_done) {
        hipEventSynchronize(c->recv_done);
        hipEventDestroy(c->recv_done);
    }
    if (c->h_recv) hipHostFree(c->h_recv);
    if (c->d_recv) hipFree(c->d_recv);
    if (c->d_zero) hipFree(c->d_zero);
    if (c->d_gf16_log) hipFree(c->d_gf16_log);
    if (c->d_gf16_exp) hipFree(c->d_gf16_exp);
    if (c->aux) {
        hipStreamSynchronize(c->aux);
        hipStreamDestroy(c->aux);
    }
    for (auto e : c->dep) hipEventDestroy(e);
    qf::bs_unload(c->bs);
    for (auto& p : c->prof_pending) {
        hipEventDestroy(p.a);
        hipEventDestroy(p.b);
    }
    for (auto e : c->ev_free) hipEventDestroy(e);
    for (int i = 0; i < qf_ctx::kPipe; ++i) {
        if (c->pstream[i]) {
            hipStreamSynchronize(c->pstream[i]);
            hipStreamDestroy(c->pstream[i]);
        }
        if (c->d_stage_src[i]) hipFree(c->d_stage_src[i]);
        if (c->d_stage_rep[i]) hipFree(c->d_stage_rep[i]);
        if (c->d_dstage[i]) hipFree(c->d_dstage[i]);
        for (hipEvent_t e : {c->ev_idx[i], c->ev_rows[i], c->ev_done[i]})
            if (e) hipEventDestroy(e);
    }
    if (c->own_stream && c->stream) hipStreamDestroy(c->stream);
    delete c;
    return QF_OK;
}

int qf_ctx_set_option(qf_ctx* ctx, int option, int64_t value) {
    if (!ctx || option < 0 || option >= QF_OPT_COUNT) return QF_EINVAL;
    std::lock_guard<std::mutex> g(ctx->mu);
    ctx->opt[option] = clamp_opt(option, value);
    return QF_OK;
}

int qf_ctx_get_option(qf_ctx* ctx, int option, int64_t* value) {
    if (!ctx || !value || option < 0 || option >= QF_OPT_COUNT) return QF_EINVAL;
    std::lock_guard<std::mutex> g(ctx->mu);
    *value = ctx->opt[option];
    return QF_OK;
}

int qf_ctx_set_stream(qf_ctx* ctx, void* stream) {
    if (!ctx) return QF_EINVAL;
    std::lock_guard<std::mutex> g(ctx->mu);
    if (ctx->own_stream && ctx->stream) {
        hipStreamSynchronize(ctx->stream);
        hipStreamDestroy(ctx->stream);
        ctx->own_stream = false;
    }
    if (stream == QF_STREAM_NULL) {
        ctx->stream = nullptr;
    } else if (stream) {
        ctx->stream = reinterpret_cast<hipStream_t>(stream);
    } else {
        QF_CHECK_HIP(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
        ctx->own_stream = true;
    }
    return QF_OK;
}

int qf_ctx_profile(qf_ctx* ctx, int on) {
    if (!ctx) return QF_EINVAL;
    std::lock_guard<std::mutex> g(ctx->mu);
    int s = prof_drain(ctx);
    if (s) return s;
    if (on) ctx->prof_tot.clear();
    ctx->prof = on != 0;
    return QF_OK;
}

int qf_ctx_profile_read(qf_ctx* ctx, uint32_t i, const char** name, uint32_t* launches, double* total_ms) {
    if (!ctx) return QF_EINVAL;
    std::lock_guard<std::mutex> g(ctx->mu);
    int s = prof_drain(ctx);
    if (s) return s;
    if (i >= ctx->prof_tot.size()) return QF_EINVAL;
    if (name) *name = ctx->prof_tot[i].name.c_str();
    if (launches) *launches = ctx->prof_tot[i].launches;
    if (total_ms) *total_ms = ctx->prof_tot[i].ms;
    return QF_OK;
}

void* qf_ctx_stream(qf_ctx* ctx) { return ctx ? reinterpret_cast<void*>(ctx->stream) : nullptr; }

int qf_sync(qf_ctx* ctx) {
    if (!ctx) return QF_EINVAL;
    QF_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    return QF_OK;
}

int qf_gf256_mul_slice_dev(qf_ctx* ctx, const uint8_t* a, const uint8_t* b, uint8_t* out, size_t n) {
    if (!ctx || (n && (!a || !b || !out))) return QF_EINVAL;
    if (n == 0) return QF_OK;
    std::lock_guard<std::mutex> g(ctx->mu);
    int s = ensure_device(ctx);
    if (s) return s;
    if (!aligned16(a) || !aligned16(b) || !aligned16(out)) return QF_EINVAL;
    hipEvent_t ev = prof_begin(ctx, ctx->stream);
    QF_CHECK_HIP(qf::launch_mul_slice(a, b, out, n, ctx->d_explog, ctx->num_cus, ctx->stream));
    prof_end(ctx, ctx->stream, ev, "k_mul_slice");
    return QF_OK;
}

int qf_fill_splitmix_dev(qf_ctx* ctx, uint8_t* dst, size_t n, uint64_t seed, uint64_t word_offset) {
    if (!ctx || (n && !dst)) return QF_EINVAL;
    if (n == 0) return QF_OK;
    std::lock_guard<std::mutex> g(ctx->mu);
    int s = ensure_device(ctx);
    if (s) return s;
    QF_CHECK_HIP(qf::launch_fill_splitmix(dst, n, seed, word_offset, ctx->num_cus, ctx->stream));
    return QF_OK;
}

int qf_encode_batch(qf_ctx* ctx, const qf_encode_shape* sh, uint32_t G, const uint8_t* src,
                    uint8_t* rep, const uint8_t* coeff) {
    if (!ctx || !sh) return QF_EINVAL;
    std::lock_guard<std::mutex> g(ctx->mu);
    int s = ensure_device(ctx);
    if (s) return s;
    return encode_impl(ctx, sh, G, src, rep, coeff, ctx->stream);
}

int qf_encode_batch_host(qf_ctx* ctx, const qf_encode_shape* sh, uint32_t G, const uint8_t* src,
                         uint8_t* rep, const uint8_t* coeff) {
    if (!ctx || !sh) return QF_EINVAL;
    if (G == 0 || sh->r == 0 || sh->L == 0) return QF_OK;
    if (!src || !rep) return QF_EINVAL;
    const uint32_t k = sh->k, r = sh->r, L = sh->L;
    // dense generations only: rows back to back inside a generation
    if (sh->src_gen_stride != (uint64_t)k * sh->src_row_stride ||
        sh->rep_gen_stride != (uint64_t)r * sh->rep_row_stride)
        return QF_EINVAL;
    std::lock_guard<std::mutex> g(ctx->mu);
    int s = ensure_device(ctx);
    if (s) return s;
    // ~64 MiB of source per chunk
    uint64_t per = std::max<uint64_t>(1, (64ull << 20) / std::max<uint64_t>(1, sh->src_gen_stride));
    per = std::min<uint64_t>(per, G);
    const size_t sb = per * sh->src_gen_stride, rb = per * sh->rep_gen_stride;
    if (sb > ctx->stage_src_bytes || rb > ctx->stage_rep_bytes) {
        for (int i = 0; i < qf_ctx::kPipe; ++i) {
            if (ctx->pstream[i]) QF_CHECK_HIP(hipStreamSynchronize(ctx->pstream[i]));
            if (ctx->d_stage_src[i]) hipFree(ctx->d_stage_src[i]);
            if (ctx->d_stage_rep[i]) hipFree(ctx->d_stage_rep[i]);
            ctx->d_stage_src[i] = ctx->d_stage_rep[i] = nullptr;
        }
        for (int i = 0; i < qf_ctx::kPipe; ++i) {
            if (hipMalloc(&ctx->d_stage_src[i], sb) != hipSuccess) return QF_ENOMEM;
            if (hipMalloc(&ctx->d_stage_rep[i], rb) != hipSuccess) return QF_ENOMEM;
        }
        ctx->stage_src_bytes = sb;
        ctx->stage_rep_bytes = rb;
    }
    for (int i = 0; i < qf_ctx::kPipe; ++i)
        if (!ctx->pstream[i]) QF_CHECK_HIP(hipStreamCreateWithFlags(&ctx->pstream[i], hipStreamNonBlocking));
    // Chunk c on stream c % kPipe: H2D -> encode -> D2H; chunks on different
    // streams overlap copies in both directions with the kernels.
    uint32_t c = 0;
    for (uint64_t g0 = 0; g0 < G; g0 += per, ++c) {
        const uint64_t n = std::min<uint64_t>(per, G - g0);
        hipStream_t st = ctx->pstream[c % qf_ctx::kPipe];
        uint8_t* ds = ctx->d_stage_src[c % qf_ctx::kPipe];
        uint8_t* dr = ctx->d_stage_rep[c % qf_ctx::kPipe];
        QF_CHECK_HIP(hipMemcpyAsync(ds, src + g0 * sh->src_gen_stride, n * sh->src_gen_stride,
                                    hipMemcpyHostToDevice, st));
        qf_encode_shape s2 = *sh;
        int e = encode_impl(ctx, &s2, (uint32_t)n, ds, dr, coeff, st);
        if (e != QF_OK) return e;
        QF_CHECK_HIP(hipMemcpy2DAsync(rep + g0 * sh->rep_gen_stride, sh->rep_row_stride, dr,
                                      sh->rep_row_stride, L, n * r, hipMemcpyDeviceToHost, st));
    }
    for (int i = 0; i < qf_ctx::kPipe; ++i) QF_CHECK_HIP(hipStreamSynchronize(ctx->pstream[i]));
    return QF_OK;
}

static int decode_batch_impl(qf_ctx* ctx, const qf_decode_shape* sh, uint32_t G, const uint8_t* rows,
                             const uint16_t* row_index, const uint32_t* n_rows, const uint8_t* row_coeffs,
                             uint8_t* rec, uint16_t* rec_index, uint32_t* n_rec, int32_t* status,
                             bool locked = false);

int qf_decode_batch(qf_ctx* ctx, const qf_decode_shape* sh, uint32_t G, const uint8_t* rows,
                    const uint16_t* row_index, const uint32_t* n_rows, const uint8_t* row_coeffs,
                    uint8_t* rec, uint16_t* rec_index, uint32_t* n_rec, int32_t* status) {
    if (!ctx) return QF_EINVAL;
    int s = decode_batch_impl(ctx, sh, G, rows, row_index, n_rows, row_coeffs, rec, rec_index, n_rec, status);
    std::lock_guard<std::mutex> g(ctx->mu);
    if (ctx->has_payload_stream && !ctx->payload_on_stream) {
        // a path that finished on the context's stream: the caller's stream waits for it
        hipError_t e = hipSuccess;
        if (!ctx->ev_accept) e = hipEventCreateWithFlags(&ctx->ev_accept, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventRecord(ctx->ev_accept, ctx->stream);
        if (e == hipSuccess) e = hipStreamWaitEvent(ctx->payload_stream, ctx->ev_accept, 0);
        if (e != hipSuccess && s == QF_OK) s = qf::device_fail(__FILE__, __LINE__, e);
    }
    ctx->payload_wait = nullptr;  // one decode call only, whatever its outcome
    ctx->has_payload_stream = ctx->payload_on_stream = false;
    return s;
}

int qf_ctx_set_payload_stream(qf_ctx* ctx, void* stream) {
    if (!ctx) return QF_EINVAL;
    std::lock_guard<std::mutex> g(ctx->mu);
    ctx->has_payload_stream = stream != nullptr;
    ctx->payload_stream = stream == QF_STREAM_NULL ? nullptr : reinterpret_cast<hipStream_t>(stream);
    ctx->payload_on_stream = false;
    return QF_OK;
}

int qf_ctx_set_payload_wait(qf_ctx* ctx, void* event) {
    if (!ctx) return QF_EINVAL;
    std::lock_guard<std::mutex> g(ctx->mu);
    ctx->payload_wait = reinterpret_cast<hipEvent_t>(event);
    return QF_OK;
}

// Host-memory decode: the receive side of the reference starts from UDP
// datagrams in host memory (core.rs:203-232).  Chunks of ~64 MiB of rows go
// through pipe slot c % kPipe:
//   pstream[slot]: H2D indices (+ n_rows, coefficients) -> ev_idx,
//                  H2D rows -> ev_rows
//   ctx->stream:   wait ev_idx; decode (acceptance pass at once, payload pass
//                  after ev_rows: qf_ctx_set_payload_wait) -> ev_done
//   pstream[slot]: wait ev_done; D2H recovered rows, indices, counts, status
// Every kernel runs on ctx->stream, so the decode workspace is reused in
// stream order; a slot's next H2D follows its previous D2H on the same
// stream, so the staging is never overwritten early.
static size_t al256(size_t x) { return (x + 255) & ~size_t(255); }

int qf_decode_batch_host(qf_ctx* ctx, const qf_decode_shape* sh, uint32_t G, const uint8_t* rows,
                         const uint16_t* row_index, const uint32_t* n_rows, const uint8_t* row_coeffs,
                         uint8_t* rec, uint16_t* rec_index, uint32_t* n_rec, int32_t* status) {
    if (!ctx || !sh) return QF_EINVAL;
    {   // qf_ctx_set_payload_stream applies to qf_decode_batch only
        std::lock_guard<std::mutex> g(ctx->mu);
        ctx->has_payload_stream = ctx->payload_on_stream = false;
    }
    const uint32_t k = sh->k, r = sh->r, L = sh->L, mr = sh->max_rows;
    if (k == 0 || k > 256 || mr == 0 || mr > 4096 || L == 0) return QF_EINVAL;
    if (G == 0) return QF_OK;
    const uint32_t e_max = std::min(k, r);
    if (!rows || !row_index || !n_rec || !status || (e_max && (!rec || !rec_index))) return QF_EINVAL;
    // generation g's rows lie in [g * rows_gen_stride, +rows_gen_stride);
    // recovered rows are dense per generation (copied back row by row)
    if (sh->rows_gen_stride < (uint64_t)(mr - 1) * sh->row_stride + L ||
        (e_max && sh->rec_gen_stride != (uint64_t)e_max * sh->rec_row_stride) || sh->rec_row_stride < L)
        return QF_EINVAL;
    {
        std::lock_guard<std::mutex> g(ctx->mu);
        int s = ensure_device(ctx);
        if (s) return s;
    }
    const uint64_t per_gen_in = sh->rows_gen_stride + 2ull * mr + 4 + (row_coeffs ? (uint64_t)mr * k : 0);
    uint64_t per = std::max<uint64_t>(1, (64ull << 20) / per_gen_in);
    per = std::min<uint64_t>(per, G);
    // staging layout of one slot (256-B aligned parts)
    const size_t o_rows = 0, o_idx = al256(per * sh->rows_gen_stride), o_n = o_idx + al256(per * mr * 2),
                 o_coef = o_n + al256(per * 4), o_rec = o_coef + (row_coeffs ? al256(per * mr * k) : 0),
                 o_ridx = o_rec + al256(per * sh->rec_gen_stride), o_nrec = o_ridx + al256(per * e_max * 2 + 2),
                 o_st = o_nrec + al256(per * 4), total = o_st + al256(per * 4);
    {
        std::lock_guard<std::mutex> g(ctx->mu);
        if (total > ctx->dstage_bytes) {
            for (int i = 0; i < qf_ctx::kPipe; ++i) {
                if (ctx->pstream[i]) QF_CHECK_HIP(hipStreamSynchronize(ctx->pstream[i]));
                if (ctx->d_dstage[i]) hipFree(ctx->d_dstage[i]);
                ctx->d_dstage[i] = nullptr;
            }
            QF_CHECK_HIP(hipStreamSynchronize(ctx->stream));
            ctx->dstage_bytes = 0;
            for (int i = 0; i < qf_ctx::kPipe; ++i)
                if (hipMalloc(&ctx->d_dstage[i], total) != hipSuccess) return QF_ENOMEM;
            ctx->dstage_bytes = total;
        }
        for (int i = 0; i < qf_ctx::kPipe; ++i) {
            if (!ctx->pstream[i]) QF_CHECK_HIP(hipStreamCreateWithFlags(&ctx->pstream[i], hipStreamNonBlocking));
            for (hipEvent_t* e : {&ctx->ev_idx[i], &ctx->ev_rows[i], &ctx->ev_done[i]})
                if (!*e) QF_CHECK_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
        }
    }
    int first_err = QF_OK;
    uint32_t c = 0;
    for (uint64_t g0 = 0; g0 < G; g0 += per, ++c) {
        const uint64_t n = std::min<uint64_t>(per, G - g0);
        const int slot = c % qf_ctx::kPipe;
        hipStream_t ps = ctx->pstream[slot];
        uint8_t* d = ctx->d_dstage[slot];
        QF_CHECK_HIP(hipMemcpyAsync(d + o_idx, row_index + g0 * mr, n * mr * 2, hipMemcpyHostToDevice, ps));
        if (n_rows) QF_CHECK_HIP(hipMemcpyAsync(d + o_n, n_rows + g0, n * 4, hipMemcpyHostToDevice, ps));
        if (row_coeffs)
            QF_CHECK_HIP(hipMemcpyAsync(d + o_coef, row_coeffs + g0 * mr * k, n * mr * k, hipMemcpyHostToDevice, ps));
        QF_CHECK_HIP(hipEventRecord(ctx->ev_idx[slot], ps));
        QF_CHECK_HIP(hipMemcpyAsync(d + o_rows, rows + g0 * sh->rows_gen_stride, n * sh->rows_gen_stride,
                                    hipMemcpyHostToDevice, ps));
        QF_CHECK_HIP(hipEventRecord(ctx->ev_rows[slot], ps));
        QF_CHECK_HIP(hipStreamWaitEvent(ctx->stream, ctx->ev_idx[slot], 0));
        // (row coefficients, read by the acceptance pass, landed before ev_idx)
        qf_ctx_set_payload_wait(ctx, ctx->ev_rows[slot]);
        int e = qf_decode_batch(ctx, sh, (uint32_t)n, d + o_rows, reinterpret_cast<const uint16_t*>(d + o_idx),
                                n_rows ? reinterpret_cast<const uint32_t*>(d + o_n) : nullptr,
                                row_coeffs ? d + o_coef : nullptr, e_max ? d + o_rec : nullptr,
                                e_max ? reinterpret_cast<uint16_t*>(d + o_ridx) : nullptr,
                                reinterpret_cast<uint32_t*>(d + o_nrec), reinterpret_cast<int32_t*>(d + o_st));
        if (e != QF_OK) {
            first_err = e;
            break;
        }
        QF_CHECK_HIP(hipEventRecord(ctx->ev_done[slot], ctx->stream));
        QF_CHECK_HIP(hipStreamWaitEvent(ps, ctx->ev_done[slot], 0));
        if (e_max) {
            QF_CHECK_HIP(hipMemcpy2DAsync(rec + g0 * sh->rec_gen_stride, sh->rec_row_stride, d + o_rec,
                                          sh->rec_row_stride, L, n * e_max, hipMemcpyDeviceToHost, ps));
            QF_CHECK_HIP(hipMemcpyAsync(rec_index + g0 * e_max, d + o_ridx, n * e_max * 2, hipMemcpyDeviceToHost, ps));
        }
        QF_CHECK_HIP(hipMemcpyAsync(n_rec + g0, d + o_nrec, n * 4, hipMemcpyDeviceToHost, ps));
        QF_CHECK_HIP(hipMemcpyAsync(status + g0, d + o_st, n * 4, hipMemcpyDeviceToHost, ps));
    }
    for (int i = 0; i < qf_ctx::kPipe; ++i) QF_CHECK_HIP(hipStreamSynchronize(ctx->pstream[i]));
    QF_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    return first_err;
}

// locked: the caller holds ctx->mu (qf_decode_batch_desc keeps it across its
// classes, so the offset tables it sets on the context and its metadata
// buffers cannot change under this call)
static int decode_batch_impl(qf_ctx* ctx, const qf_decode_shape* sh, uint32_t G, const uint8_t* rows,
                             const uint16_t* row_index, const uint32_t* n_rows, const uint8_t* row_coeffs,
                             uint8_t* rec, uint16_t* rec_index, uint32_t* n_rec, int32_t* status,
                             bool locked) {
    if (!ctx || !sh) return QF_EINVAL;
    const uint32_t k = sh->k, r = sh->r, L = sh->L, max_rows = sh->max_rows;
    if (k == 0 || k > 256 || max_rows == 0 || max_rows > 4096 || L == 0) return QF_EINVAL;
    if (G == 0) return QF_OK;
    if (!rows || !row_index || !n_rec || !status) return QF_EINVAL;
    const uint32_t e_max = std::min(k, r);
    if (e_max > 128) return QF_EINVAL;
    if (e_max && (!rec || !rec_index)) return QF_EINVAL;
    if (!aligned16(rows) || (sh->row_stride & 15) || (sh->rows_gen_stride & 15)) return QF_EINVAL;
    if (e_max && (!aligned16(rec) || (sh->rec_row_stride & 15) || (sh->rec_gen_stride & 15)))
        return QF_EINVAL;
    std::unique_lock<std::mutex> g(ctx->mu, std::defer_lock);
    if (!locked) g.lock();
    int s = ensure_device(ctx);
    if (s) return s;
    if (!row_coeffs && ctx->opt[QF_OPT_BITSLICED] && r <= 16 && k + r <= 256 && qf::syn_available(k, r) &&
        max_rows <= 255 && L >= 32 && sh->rows_gen_stride < (1ull << 32) &&
        sh->row_stride < (1ull << 32) && (uint64_t)G * qf::bs_padded_units(L) < (1ull << 31) &&
        (uint64_t)r * 16 * qf::bs_padded_units(L) < (1ull << 32)) {
        // fused single-pass decode unless QF_DECODE_SYN=1 asks for the
        // two-kernel syndrome + v_perm combine path
        const bool two = ctx->opt[QF_OPT_DECODE_PATH] == 1;
        // (L % 16 != 0: the lane-chunk kernel stores the partial last unit
        // bytewise but reads it whole, so the rows must start 16-byte aligned;
        // a desc batch's offset tables say so through offs_in_al16)
        const bool tail_ok = L % 16 == 0 || (qf::dec_name(&ctx->bs, k, r, L) && (!ctx->offs_in || ctx->offs_in_al16) &&
                                             ((uintptr_t)rows | sh->row_stride |
                                              (ctx->offs_in ? 0 : sh->rows_gen_stride)) % 16 == 0 &&
                                             std::string(qf::dec_name(&ctx->bs, k, r, L)).find("decc") != std::string::npos);
        // (the row-split 'decs' kernels of small batches share the decc layout)
        if (qf::dec_available(k, r) && !two && tail_ok && sh->rec_gen_stride < (1ull << 32) &&
            sh->rec_row_stride < (1ull << 32))
            return decode_fused(ctx, sh, G, rows, row_index, n_rows, rec, rec_index, n_rec, status);
        return decode_cauchy(ctx, sh, G, rows, row_index, n_rows, rec, rec_index, n_rec, status);
    }
    // codes without a syndrome kernel but with encode kernels (C5 Medium
    // windows: r up to 64): syndromes through the encode kernels
    if (!row_coeffs && ctx->opt[QF_OPT_BITSLICED] && !qf::syn_available(k, r) && qf::bs_available(k, r) && r <= 64 &&
        e_max <= 64 && k + r <= 256 && max_rows <= 255 && L >= 32 && sh->rows_gen_stride < (1ull << 32) &&
        sh->row_stride < (1ull << 32) && (uint64_t)G * qf::bs_padded_units(L) < (1ull << 31))
        return decode_cauchy_enc(ctx, sh, G, rows, row_index, n_rows, rec, rec_index, n_rec, status);
    const uint32_t passes = (e_max + 15) / 16;
    const uint64_t coef_gen_stride = ((uint64_t)max_rows + 1) * 16;
    const size_t coef_bytes = (size_t)std::max<uint32_t>(passes, 1) * G * coef_gen_stride;
    const size_t bound_off = round_up(coef_bytes, 256);
    s = grow_work(ctx, bound_off + (size_t)G * 4);
    if (s) return s;
    uint8_t* d_coef = ctx->d_work;
    uint32_t* d_bound = reinterpret_cast<uint32_t*>(ctx->d_work + bound_off);
    qf::PrepareArgs pa{};
    pa.row_index = row_index;
    pa.n_rows = n_rows;
    pa.row_coeffs = row_coeffs;
    pa.explog = ctx->d_explog;
    pa.coef_out = d_coef;
    pa.coef_gen_stride = coef_gen_stride;
    pa.n_out = n_rec;
    pa.bound = d_bound;
    pa.rec_index = rec_index;
    pa.status = status;
    pa.k = k;
    pa.e_max = e_max;
    pa.e_lds = std::min<uint32_t>(k, 128);
    pa.rep_limit = row_coeffs ? 256 : r;
    pa.max_rows = max_rows;
    pa.max_rows_pad = (max_rows + 7) & ~7u;
    pa.passes = passes;
    pa.G = G;
    if (qf::prepare_lds_bytes(k, pa.e_lds, max_rows) > 160 * 1024) return QF_EINVAL;
    hipEvent_t ev = prof_begin(ctx, ctx->stream);
    QF_CHECK_HIP(qf::launch_decode_prepare(pa, ctx->stream));
    prof_end(ctx, ctx->stream, ev, "k_decode_prepare");
    if (int gs = payload_gate(ctx, ctx->stream)) return gs;
    const uint32_t Lu = (L + 15) / 16;
    bool pm = false;   // every pass in one pass-major launch, as in decode_cauchy_syn
    for (uint32_t p = 0; p < passes && !pm; ++p) {
        qf::CombineSlotsArgs a{};
        a.rows = rows;
        a.rows_gen_stride = sh->rows_gen_stride;
        a.rows_offs = ctx->offs_in;
        a.dst_offs = ctx->offs_out;
        a.row_stride = sh->row_stride;
        a.dst = rec + (uint64_t)p * 16 * sh->rec_row_stride;
        a.dst_gen_stride = sh->rec_gen_stride;
        a.dst_row_stride = sh->rec_row_stride;
        a.coef = d_coef + (uint64_t)p * G * coef_gen_stride;
        a.coef_gen_stride = coef_gen_stride;
        a.n_out = n_rec;
        a.bound = d_bound;
        a.tab256 = ctx->d_tab256;
        a.pass = p;
        a.L = L;
        a.Lu = Lu;
        a.zero_slot = max_rows;
        a.total_units = (uint64_t)G * Lu;
        const int PD = pick_PD(ctx, QF_OPT_DECODE_PD, 1);
        hipEvent_t ev2 = prof_begin(ctx, ctx->stream);
        std::string cname;
        // (at most kCmbMaxPasses passes per launch: e_max reaches 128 on this
        // path, i.e. up to 8 passes, which then run one launch per pass)
        pm = p == 0 && ctx->opt[QF_OPT_ENCODE_MERGED] &&
             qf::cmb_pass_major_ok(passes, sh->rec_row_stride, (uint64_t)G * coef_gen_stride) &&
             combine_bs_ok(ctx, a, a.rows_offs == ctx->offs_in && ctx->offs_in_al16);
        if (pm) {
            cname = qf::cmb_kernel_name(ctx->bs, a, passes, (uint64_t)G * coef_gen_stride, e_max);
            QF_CHECK_HIP(qf::cmb_launch(ctx->bs, ctx->num_cus, ctx->stream, a, ctx->d_cmbidx, passes,
                                        (uint64_t)G * coef_gen_stride, e_max));
        } else {
            QF_CHECK_HIP(combine_payload(ctx, a, PD, ctx->stream, &cname));
        }
        prof_end(ctx, ctx->stream, ev2, cname);
    }
    return QF_OK;
}

int qf_frame_batch_dev(qf_ctx* ctx, const qf_encode_shape* sh, uint32_t G, const uint8_t* src,
                       const uint8_t* rep, uint8_t* frames, uint64_t frame_stride, uint32_t* frame_len) {
    if (!ctx || !sh) return QF_EINVAL;
    const uint32_t k = sh->k, r = sh->r, L = sh->L;
    if (k == 0 || k + r > 256) return k == 0 ? QF_EINVAL : QF_ERANGE;
    if (G == 0 || L == 0) return QF_OK;
    if (!src || !frames || (r && !rep)) return QF_EINVAL;
    if (frame_stride < 3ull + k + L || (frame_stride & 15) || !aligned16(frames)) return QF_EINVAL;
    if (!aligned16(src) || (sh->src_row_stride & 15) || (sh->src_gen_stride & 15)) return QF_EINVAL;
    if (r && (!aligned16(rep) || (sh->rep_row_stride & 15) || (sh->rep_gen_stride & 15))) return QF_EINVAL;
    std::lock_guard<std::mutex> g(ctx->mu);
    int s = ensure_device(ctx);
    if (s) return s;
    hipEvent_t ev = prof_begin(ctx, ctx->stream);
    QF_CHECK_HIP(qf::launch_frame_batch(src, rep, *sh, G, frames, frame_stride, frame_len, ctx->d_explog,
                                        ctx->num_cus, ctx->stream));
    prof_end(ctx, ctx->stream, ev, "k_frame_batch");
    return QF_OK;
}

int qf_parse_frames_dev(qf_ctx* ctx, uint32_t k, uint32_t r, uint32_t L, uint32_t G, uint32_t max_rows,
                        const uint8_t* frames, uint64_t frame_stride, const uint32_t* frame_len,
                        const uint64_t* ids, const uint32_t* n_frames, uint8_t* rows, uint64_t row_stride,
                        uint64_t rows_gen_stride, uint16_t* row_index, uint32_t* n_rows, int32_t* frame_status) {
    if (!ctx) return QF_EINVAL;
    if (k == 0 || k + r > 256) return k == 0 ? QF_EINVAL : QF_ERANGE;
    if (G == 0) return QF_OK;
    if (max_rows == 0 || max_rows > 1024 || L == 0) return QF_EINVAL;
    if (!frames || !frame_len || !ids || !rows || !row_index || !n_rows || !frame_status) return QF_EINVAL;
    if ((frame_stride & 15) || !aligned16(frames) || !aligned16(rows) || (row_stride & 15) ||
        (rows_gen_stride & 15) || row_stride < L)
        return QF_EINVAL;
    std::lock_guard<std::mutex> g(ctx->mu);
    int s = ensure_device(ctx);
    if (s) return s;
    hipEvent_t ev = prof_begin(ctx, ctx->stream);
    QF_CHECK_HIP(qf::launch_parse_frames(frames, frame_stride, frame_len, ids, n_frames, k, r, L, G, max_rows, rows,
                                         row_stride, rows_gen_stride, row_index, n_rows, frame_status,
                                         ctx->d_explog, ctx->stream));
    prof_end(ctx, ctx->stream, ev, "k_parse_frames");
    return QF_OK;
}


// ---------------------------------------------------------------------------
// Heterogeneous batches (SURVEY 8(b) qf_gen_desc): one call over generations
// of different (k, r, L) at arbitrary offsets.  Generations are grouped by
// shape; each class runs the batch implementation above with per-generation
// offset tables (every kernel addresses generation g at base + table[g]).
// ---------------------------------------------------------------------------
namespace {

// pinned staging (reused per call: the previous upload must have landed)
int desc_stage(qf_ctx* ctx, size_t bytes) {
    if (!ctx->desc_done) QF_CHECK_HIP(hipEventCreateWithFlags(&ctx->desc_done, hipEventDisableTiming));
    else QF_CHECK_HIP(hipEventSynchronize(ctx->desc_done));
    if (bytes > ctx->h_desc_bytes) {
        if (ctx->h_desc) hipHostFree(ctx->h_desc);
        ctx->h_desc = nullptr;
        ctx->h_desc_bytes = 0;
        const size_t b = round_up(bytes, 1 << 16);
        if (hipHostMalloc(reinterpret_cast<void**>(&ctx->h_desc), b) != hipSuccess) return QF_ENOMEM;
        ctx->h_desc_bytes = b;
    }
    if (bytes > ctx->desc_bytes) {
        if (ctx->d_desc) {
            QF_CHECK_HIP(hipStreamSynchronize(ctx->stream));
            hipFree(ctx->d_desc);
        }
        ctx->d_desc = nullptr;
        ctx->desc_bytes = 0;
        const size_t b = round_up(bytes, 1 << 16);
        if (hipMalloc(&ctx->d_desc, b) != hipSuccess) return QF_ENOMEM;
        ctx->desc_bytes = b;
    }
    return QF_OK;
}

int desc_upload(qf_ctx* ctx, size_t bytes) {
    QF_CHECK_HIP(hipMemcpyAsync(ctx->d_desc, ctx->h_desc, bytes, hipMemcpyHostToDevice, ctx->stream));
    QF_CHECK_HIP(hipEventRecord(ctx->desc_done, ctx->stream));
    return QF_OK;
}

struct OffsScope {  // the class's offset tables for the launches inside the batch implementation
    qf_ctx* ctx;
    OffsScope(qf_ctx* c, const uint64_t* in, const uint64_t* out) : ctx(c) {
        ctx->offs_in = in;
        ctx->offs_out = out;
    }
    ~OffsScope() {
        ctx->offs_in = nullptr;
        ctx->offs_out = nullptr;
    }
};

}  // namespace

int qf_encode_batch_desc(qf_ctx* ctx, const qf_gen_desc* gens, uint32_t G, const uint8_t* src, uint8_t* rep) {
    if (!ctx) return QF_EINVAL;
    if (G == 0) return QF_OK;
    if (!gens || !src || !rep || !aligned16(src) || !aligned16(rep)) return QF_EINVAL;
    typedef std::tuple<uint32_t, uint32_t, uint32_t, uint32_t, uint64_t, uint64_t> Key;
    std::map<Key, std::vector<uint32_t>> cls;
    for (uint32_t i = 0; i < G; ++i) {
        const qf_gen_desc& d = gens[i];
        if (d.k == 0 || d.k > 256 || (d.flags & ~QF_ENCODE_ZERO_TAIL)) return QF_EINVAL;
        if (d.k + d.r > 256) return QF_ERANGE;  // gf_inv(0) in the Cauchy rows (decoder.rs:290-296)
        if (d.r == 0 || d.L == 0) continue;      // nothing to emit
        if ((d.src_offset | d.src_row_stride | d.rep_offset | d.rep_row_stride) & 15) return QF_EINVAL;
        if ((d.src_row_stride < d.L && d.k > 1) || (d.rep_row_stride < d.L && d.r > 1)) return QF_EINVAL;
        cls[Key(d.k, d.r, d.L, d.flags, d.src_row_stride, d.rep_row_stride)].push_back(i);
    }
    std::lock_guard<std::mutex> g(ctx->mu);
    int s = ensure_device(ctx);
    if (s) return s;
    size_t n = 0;
    for (auto& kv : cls) n += kv.second.size();
    if (n == 0) return QF_OK;
    if ((s = desc_stage(ctx, 16 * n)) != QF_OK) return s;
    uint64_t* h = reinterpret_cast<uint64_t*>(ctx->h_desc);
    size_t o = 0;
    for (auto& kv : cls) {   // per class: source offsets, then repair offsets
        for (uint32_t i : kv.second) h[o++] = gens[i].src_offset;
        for (uint32_t i : kv.second) h[o++] = gens[i].rep_offset;
    }
    if ((s = desc_upload(ctx, 16 * n)) != QF_OK) return s;
    const uint64_t* dt = reinterpret_cast<const uint64_t*>(ctx->d_desc);
    o = 0;
    for (auto& kv : cls) {
        const uint32_t Gc = (uint32_t)kv.second.size();
        qf_encode_shape sh{};
        std::tie(sh.k, sh.r, sh.L, sh.flags, sh.src_row_stride, sh.rep_row_stride) = kv.first;
        OffsScope scope(ctx, dt + o, dt + o + Gc);
        s = encode_impl(ctx, &sh, Gc, src, rep, nullptr, ctx->stream);
        if (s != QF_OK) return s;
        o += 2 * (size_t)Gc;
    }
    return QF_OK;
}

int qf_decode_batch_desc(qf_ctx* ctx, const qf_dec_desc* gens, uint32_t G, const uint8_t* rows,
                         const uint16_t* row_index, uint8_t* rec, uint16_t* rec_index, uint32_t* n_rec,
                         int32_t* status) {
    if (!ctx) return QF_EINVAL;
    {   // qf_ctx_set_payload_stream applies to qf_decode_batch only
        std::lock_guard<std::mutex> g(ctx->mu);
        ctx->has_payload_stream = ctx->payload_on_stream = false;
    }
    if (G == 0) return QF_OK;
    if (!gens || !rows || !row_index || !n_rec || !status || !aligned16(rows)) return QF_EINVAL;
    typedef std::tuple<uint32_t, uint32_t, uint32_t, uint64_t, uint64_t> Key;
    std::map<Key, std::vector<uint32_t>> cls;
    bool any_rec = false;
    for (uint32_t i = 0; i < G; ++i) {
        const qf_dec_desc& d = gens[i];
        if (d.k == 0 || d.k > 256 || d.L == 0 || d.n_rows > 255) return QF_EINVAL;
        if (std::min(d.k, d.r) > 128) return QF_EINVAL;
        if ((d.rows_offset | d.row_stride | d.rec_offset | d.rec_row_stride) & 15) return QF_EINVAL;
        if (d.row_stride < d.L && d.n_rows > 1) return QF_EINVAL;
        any_rec = any_rec || std::min(d.k, d.r) > 0;
        cls[Key(d.k, d.r, d.L, d.row_stride, d.rec_row_stride)].push_back(i);
    }
    if (any_rec && (!rec || !rec_index || !aligned16(rec))) return QF_EINVAL;
    int s;
    // metadata per generation (class order): rows / rec offset tables (8 + 8),
    // row-index / rec-index element offsets (8 + 8), n_rows and descriptor id
    // (4 + 4); per class also the gathered row indices, n_rows, and the
    // class's recovered indices, counts and statuses before the scatter
    size_t meta = 0, scratch = 0;
    std::vector<size_t> cls_scratch;
    for (auto& kv : cls) {
        const uint32_t Gc = (uint32_t)kv.second.size(), k = std::get<0>(kv.first), r = std::get<1>(kv.first);
        uint32_t mr = 1;
        for (uint32_t i : kv.second) mr = std::max(mr, gens[i].n_rows);
        const size_t emax = std::min(k, r);
        meta += 40 * (size_t)Gc;
        cls_scratch.push_back(scratch);
        scratch += round_up((size_t)Gc * mr * 2, 256) + round_up((size_t)Gc * emax * 2, 256) + round_up((size_t)Gc * 12, 256);
    }
    // one lock for the staging and every class: the offset tables set on the
    // context and the metadata buffers stay this call's until it returns
    std::lock_guard<std::mutex> lk(ctx->mu);
    {
        if ((s = ensure_device(ctx)) != QF_OK) return s;
        if ((s = desc_stage(ctx, round_up(meta, 256) + scratch)) != QF_OK) return s;
        uint8_t* h = ctx->h_desc;
        size_t o = 0;
        for (auto& kv : cls) {
            const size_t Gc = kv.second.size();
            uint64_t* ro = reinterpret_cast<uint64_t*>(h + o);
            uint64_t* co = ro + Gc;
            uint64_t* rio = co + Gc;
            uint64_t* cio = rio + Gc;
            uint32_t* nr = reinterpret_cast<uint32_t*>(cio + Gc);
            uint32_t* id = nr + Gc;
            for (size_t q = 0; q < Gc; ++q) {
                const qf_dec_desc& d = gens[kv.second[q]];
                ro[q] = d.rows_offset;
                co[q] = d.rec_offset;
                rio[q] = d.row_index_offset;
                cio[q] = d.rec_index_offset;
                nr[q] = d.n_rows;
                id[q] = kv.second[q];
            }
            o += 40 * Gc;
        }
        if ((s = desc_upload(ctx, meta)) != QF_OK) return s;
    }
    uint8_t* dm = ctx->d_desc;
    uint8_t* dsc = ctx->d_desc + round_up(meta, 256);
    size_t o = 0, c = 0;
    for (auto& kv : cls) {
        const uint32_t Gc = (uint32_t)kv.second.size();
        qf_decode_shape sh{};
        std::tie(sh.k, sh.r, sh.L, sh.row_stride, sh.rec_row_stride) = kv.first;
        uint32_t mr = 1;
        for (uint32_t i : kv.second) mr = std::max(mr, gens[i].n_rows);
        const uint32_t emax = std::min(sh.k, sh.r);
        sh.max_rows = mr;
        const uint64_t* ro = reinterpret_cast<const uint64_t*>(dm + o);
        const uint64_t* co = ro + Gc;
        const uint64_t* rio = co + Gc;
        const uint64_t* cio = rio + Gc;
        const uint32_t* nr = reinterpret_cast<const uint32_t*>(cio + Gc);
        const uint32_t* id = nr + Gc;
        uint8_t* sc = dsc + cls_scratch[c];
        uint16_t* ri_ws = reinterpret_cast<uint16_t*>(sc);
        uint16_t* rec_ws = reinterpret_cast<uint16_t*>(sc + round_up((size_t)Gc * mr * 2, 256));
        uint32_t* nrec_ws = reinterpret_cast<uint32_t*>(sc + round_up((size_t)Gc * mr * 2, 256) +
                                                        round_up((size_t)Gc * emax * 2, 256));
        int32_t* st_ws = reinterpret_cast<int32_t*>(nrec_ws + Gc);
        {
            qf::DescIndexArgs ia{row_index, rio, nr, ri_ws, mr, Gc};
            QF_CHECK_HIP(qf::launch_desc_gather_index(ia, ctx->stream));
            ctx->offs_in = ro;
            ctx->offs_out = co;
            bool al = ((uintptr_t)rows % 16) == 0;
            for (uint32_t i : kv.second) al = al && gens[i].rows_offset % 16 == 0;
            ctx->offs_in_al16 = al;
        }
        s = decode_batch_impl(ctx, &sh, Gc, rows, ri_ws, nr, nullptr, rec, rec_ws, nrec_ws, st_ws, true);
        ctx->offs_in = ctx->offs_out = nullptr;
        ctx->offs_in_al16 = false;
        if (s != QF_OK) {
            ctx->payload_wait = nullptr;
            return s;
        }
        qf::DescOutArgs oa{rec_ws, nrec_ws, st_ws, cio, id, rec_index, n_rec, status, emax, Gc};
        QF_CHECK_HIP(qf::launch_desc_scatter_out(oa, ctx->stream));
        o += 40 * (size_t)Gc;
        ++c;
    }
    ctx->payload_wait = nullptr;  // as qf_decode_batch: one decode call only
    return QF_OK;
}

int qf_selftest_split_tables(void) {
    const auto& f = gf();
    uint32_t rec[8];
    for (int c = 0; c < 256; ++c) {
        qf::perm_record((uint8_t)c, rec);
        for (int x = 0; x < 256; x += 4) {
            const uint32_t packed = qf::pack4((uint8_t)x, (uint8_t)(x + 1), (uint8_t)(x + 2), (uint8_t)(x + 3));
            const uint32_t got = qf::perm_mul4_emul(rec, packed);
            for (int b = 0; b < 4; ++b)
                if (((got >> (8 * b)) & 0xFF) != f.mul((uint8_t)c, (uint8_t)(x + b))) return QF_EINVAL;
        }
    }
    return QF_OK;
}

// ---------------------------------------------------------------------------
// Wire framing (encoder.rs:18-152)
// ---------------------------------------------------------------------------
int qf_packet_to_raw(int is_systematic, const uint8_t* coeffs, uint32_t coeff_len,
                     const uint8_t* payload, uint32_t len, uint8_t* out, uint32_t out_cap,
                     uint32_t* out_len) {
    if (!out || !out_len || (len && !payload) || coeff_len > 0xFFFF) return QF_EINVAL;
    uint64_t need = (uint64_t)len + 1 + (coeffs ? 2 + (uint64_t)coeff_len : 0);
    if (need > out_cap) return QF_ETOOSMALL;
    uint32_t o = 0;
    out[o++] = is_systematic ? 1 : 0;
    if (coeffs) {
        out[o++] = (uint8_t)(coeff_len >> 8);
        out[o++] = (uint8_t)(coeff_len & 0xFF);
        memcpy(out + o, coeffs, coeff_len);
        o += coeff_len;
    }
    if (len) memcpy(out + o, payload, len);
    o += len;
    *out_len = o;
    return QF_OK;
}

int qf_packet_from_raw(const uint8_t* raw, uint32_t raw_len, int* is_systematic,
                       const uint8_t** coeffs, uint32_t* coeff_len, const uint8_t** payload,
                       uint32_t* len) {
    if (!is_systematic || !coeffs || !coeff_len || !payload || !len) return QF_EINVAL;
    if (!raw || raw_len == 0) return QF_EINVAL;  // "Raw data is empty"
    const int sys = raw[0] == 1;
    uint32_t off = 1;
    *coeffs = nullptr;
    *coeff_len = 0;
    if (!sys) {
        if (raw_len < 3) return QF_ETOOSMALL;  // coefficient length missing
        const uint32_t cl = ((uint32_t)raw[1] << 8) | raw[2];
        off = 3;
        if (raw_len < off + cl) return QF_ETOOSMALL;  // coefficients truncated
        *coeffs = raw + off;
        *coeff_len = cl;
        off += cl;
    }
    *is_systematic = sys;
    *payload = raw + off;
    *len = raw_len - off;
    return QF_OK;
}

int qf_packet_from_block(uint8_t* block, uint32_t block_len, uint32_t len, int* is_systematic,
                         uint8_t* coeffs_out, uint32_t coeffs_cap, uint32_t* coeff_len, uint32_t* payload_len) {
    if (!block || !is_systematic || !coeff_len || !payload_len) return QF_EINVAL;
    if (len == 0 || len > block_len) return QF_EINVAL;  // "Invalid raw packet length" (encoder.rs:78-82)
    const int sys = block[0] == 1;
    uint32_t off = 1, cl = 0;
    if (!sys) {
        if (len < 3) return QF_ETOOSMALL;  // coefficient length missing (encoder.rs:88-92)
        cl = ((uint32_t)block[1] << 8) | block[2];
        off = 3;
        if (len < off + cl) return QF_ETOOSMALL;  // coefficients truncated (encoder.rs:95-99)
        if (cl > block_len || cl > coeffs_cap || (cl && !coeffs_out)) return QF_ETOOSMALL;
        if (cl) memcpy(coeffs_out, block + off, cl);
        off += cl;
    }
    memmove(block, block + off, len - off);  // copy_within(payload_offset..len, 0) (encoder.rs:108-110)
    *is_systematic = sys;
    *coeff_len = cl;
    *payload_len = len - off;
    return QF_OK;
}

}  // extern "C"
