// qf_adaptive.hip -- the adaptive sliding-window FEC driver of the C ABI
// (include/qf_fec.h, "Adaptive FEC driver").
//
// A restatement of the reference's controller and its per-connection codec
// plumbing (adaptive.rs:44-631, mod.rs:56-79, decoder.rs:90-153) over the
// GF(2^8) encoder / decoder objects of qf_objects.hip and, in Extreme mode,
// the GF(2^16) ones of qf_objects16.hip.  Host logic only: the payload
// arithmetic runs in the objects' device kernels.
//
// Arithmetic is f32 and evaluated operation by operation as Rust does (no
// FMA contraction), so mode and window decisions match the reference for the
// same loss reports and clock readings.  Reference defects are kept, because
// a drop-in must decide as the reference decides:
//  * the PID error is setpoint - measured loss, so heavy loss drives the
//    output negative and steps the mode down (adaptive.rs:215-223, 306);
//  * the 500 ms dwell check precedes the PID, so only the emergency override
//    can change the mode in the first 500 ms (adaptive.rs:199-201);
//  * report_loss without a mode/window change rebuilds the codec, dropping
//    the window (adaptive.rs:626-629).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <deque>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "qf_fec.h"
#include "qf_internal.h"

#pragma clang fp contract(off)

namespace {

double monotonic_s() {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + (double)ts.tv_nsec * 1e-9;
}

// Duration::as_secs_f32 of (now - then)
float secs_f32(double now, double then) {
    double d = now - then;
    if (d < 0) d = 0;
    return (float)d;
}

// f32 -> usize as Rust's saturating `as` cast
uint32_t sat_u32(float x) {
    if (!(x > 0.0f)) return 0;  // negative and NaN -> 0
    if (x >= 4294967295.0f) return 0xFFFFFFFFu;
    return (uint32_t)x;
}

const float kThreshold[6] = {0.01f, 0.05f, 0.15f, 0.30f, 0.50f, 1.0f};  // adaptive.rs:161-166
const float kRatio[6] = {1.0f, 1.05f, 1.15f, 1.30f, 1.50f, 2.0f};       // adaptive.rs:135-147
const uint32_t kRangeLo[6] = {0, 8, 32, 64, 256, 1024};                 // adaptive.rs:124-133
const uint32_t kRangeHi[6] = {0, 32, 128, 256, 1024, 4096};
const float kMinDwell = 0.5f;   // adaptive.rs:181
const float kAlphaK = 0.5f;     // adaptive.rs:115
const uint32_t kFade = QF_CROSS_FADE_LEN;

bool mode_ok(int32_t m) { return m >= QF_MODE_ZERO && m <= QF_MODE_EXTREME; }

// mod.rs:56-79
struct Kalman {
    float estimate = 0.0f, error_cov = 1.0f, q = 0.0f, r = 0.0f;
    float update(float m) {
        error_cov += q;
        const float k = error_cov / (error_cov + r);
        estimate += k * (m - estimate);
        error_cov *= 1.0f - k;
        return estimate;
    }
};

// adaptive.rs:44-99
struct LossEstimator {
    float ema = 0.0f, lambda = 0.1f;
    std::deque<bool> window;
    uint32_t capacity = 20;
    bool use_kalman = false;
    Kalman kf;

    void report(uint32_t lost, uint32_t total) {
        float cur = total > 0 ? (float)lost / (float)total : 0.0f;
        if (use_kalman) cur = kf.update(cur);
        ema = (lambda * cur) + (1.0f - lambda) * ema;
        auto push = [&](bool v) {
            if (window.size() == capacity) window.pop_front();
            window.push_back(v);
        };
        for (uint32_t i = 0; i < lost; ++i) push(true);
        for (uint32_t i = 0; i < total - lost; ++i) push(false);
    }
    float estimate() const {
        float burst = 0.0f;
        if (!window.empty()) {
            uint32_t c = 0;
            for (bool v : window) c += v ? 1 : 0;
            burst = (float)c / (float)window.size();
        }
        return ema > burst ? ema : burst;  // f32::max (no NaNs here)
    }
};

// adaptive.rs:282-324
struct Pid {
    float kp = 0, ki = 0, kd = 0, integral = 0, prev_error = 0;
    double last_time = 0;
    float update(float current, float setpoint, double now) {
        const float dt = secs_f32(now, last_time);
        last_time = now;
        if (dt <= 0.0f) return 0.0f;
        const float error = setpoint - current;
        integral += error * dt;
        const float derivative = (error - prev_error) / dt;
        prev_error = error;
        return (kp * error) + (ki * integral) + (kd * derivative);
    }
};

int32_t next_mode(int32_t m) { return m >= QF_MODE_STRONG ? QF_MODE_EXTREME : m + 1; }
int32_t prev_mode(int32_t m) { return m <= QF_MODE_LIGHT ? QF_MODE_ZERO : m - 1; }

// adaptive.rs:102-279
struct ModeManager {
    int32_t mode = QF_MODE_ZERO;
    uint32_t window = 0;
    uint32_t windows[6] = {0, 16, 64, 128, 512, 1024};
    double last_change = 0;
    float hysteresis = 0.02f;
    Pid pid;

    // returns true (and the previous mode/window) when a cross-fade starts
    bool update(float est, double now, int32_t* pm, uint32_t* pw) {
        if (est > kThreshold[QF_MODE_STRONG] + hysteresis) {  // emergency override
            *pm = mode;
            *pw = window;
            mode = QF_MODE_EXTREME;
            window = windows[mode];
            last_change = now;
            return true;
        }
        if (secs_f32(now, last_change) < kMinDwell) return false;
        const float out = pid.update(est, kThreshold[mode], now);
        int32_t nm = mode;
        if (out > 0.1f) nm = next_mode(mode);
        else if (out < -0.1f) nm = prev_mode(mode);
        const int32_t old_mode = mode;
        const uint32_t old_window = window;
        if (nm != mode) {
            mode = nm;
            last_change = now;
            window = windows[nm];
        }
        const float alpha = 1.0f + kAlphaK * (est - kThreshold[mode]);
        uint32_t nw = sat_u32(roundf((float)window * alpha));
        if (nw < kRangeLo[mode]) nw = kRangeLo[mode];
        if (nw > kRangeHi[mode]) nw = kRangeHi[mode];
        window = nw;
        if (old_mode != mode || old_window != window) {
            *pm = old_mode;
            *pw = old_window;
            return true;
        }
        return false;
    }
};

void params_for(int32_t mode, uint32_t window, uint32_t* k, uint32_t* n) {
    *k = window;
    *n = sat_u32(ceilf((float)window * kRatio[mode]));
}

// EncoderVariant / DecoderVariant (decoder.rs:90-153): GF(2^16) objects in
// Extreme mode, GF(2^8) otherwise
struct Codec {
    int32_t mode = QF_MODE_ZERO;
    uint32_t k = 0, n = 0;
    qf_encoder* enc = nullptr;
    qf_decoder* dec = nullptr;
    qf_encoder16* enc16 = nullptr;
    qf_decoder16* dec16 = nullptr;
    int status = QF_OK;  // QF_ERANGE: the field cannot realise (mode, k, n)
    bool decoded = false;

    bool has_enc() const { return enc || enc16; }
    uint32_t coeff_bytes() const { return enc16 ? 2 * k : k; }
    void release() {
        if (enc) qf_encoder_free(enc);
        if (dec) qf_decoder_free(dec);
        if (enc16) qf_encoder16_free(enc16);
        if (dec16) qf_decoder16_free(dec16);
        enc = nullptr;
        dec = nullptr;
        enc16 = nullptr;
        dec16 = nullptr;
    }
};

}  // namespace

struct qf_adaptive {
    qf_ctx* ctx = nullptr;
    qf_fec_config cfg{};
    LossEstimator est;
    ModeManager mgr;
    Codec cur, fade;
    bool has_fade = false;
    uint32_t transition_left = 0;
    std::vector<uint8_t> scratch;
};

namespace {

int make_codec(qf_adaptive* a, int32_t mode, uint32_t k, uint32_t n, Codec* c) {
    c->mode = mode;
    c->k = k;
    c->n = n;
    c->enc = nullptr;
    c->dec = nullptr;
    c->enc16 = nullptr;
    c->dec16 = nullptr;
    c->decoded = false;
    c->status = QF_OK;
    if (k == 0) return QF_OK;  // Zero mode: nothing to encode or decode
    if (mode == QF_MODE_EXTREME) {
        // decoder.rs:96-102: GF(2^16); repairs 0..n-k need k + (n - k) <= 65536
        if (k > 4096 || n > 65536) {
            c->status = QF_ERANGE;
            return QF_OK;
        }
        if (!a->ctx) return QF_OK;
        int s = qf_encoder16_new(a->ctx, k, n, a->cfg.max_len, &c->enc16);
        if (s == QF_OK) s = qf_decoder16_new(a->ctx, k, a->cfg.max_len, &c->dec16);
        if (s != QF_OK) {
            c->release();
            return s;
        }
        return QF_OK;
    }
    if (k > 255 || n > 256) {
        c->status = QF_ERANGE;
        return QF_OK;
    }
    if (!a->ctx) return QF_OK;  // controller only
    int s = qf_encoder_new(a->ctx, k, n, a->cfg.max_len, &c->enc);
    if (s == QF_OK) s = qf_decoder_new(a->ctx, k, a->cfg.max_len, &c->dec);
    if (s != QF_OK) {
        c->release();
        return s;
    }
    return QF_OK;
}

int add_source(Codec& c, uint64_t id, const uint8_t* data, uint32_t len) {
    if (c.enc16) return qf_encoder16_add_source_packet(c.enc16, id, data, len);
    if (c.enc) return qf_encoder_add_source_packet(c.enc, id, data, len);
    return QF_OK;
}

// emit_repairs (adaptive.rs:546-562): repairs 0..n-k of a full window
int emit_repairs(Codec& c, uint8_t* out_data, uint32_t out_stride, uint8_t* out_coeffs,
                 uint32_t coeff_stride, qf_packet_desc* desc, uint32_t* n) {
    if (!c.has_enc()) return QF_OK;
    const uint32_t r = c.n - c.k;
    if (r == 0) return QF_OK;
    std::vector<uint32_t> lens(r);
    std::vector<uint64_t> ids(r);
    uint8_t* co = out_coeffs ? out_coeffs + (size_t)*n * coeff_stride : nullptr;
    int s = c.enc16 ? qf_encoder16_generate_repairs(c.enc16, 0, r, out_data + (size_t)*n * out_stride, out_stride,
                                                    lens.data(), co, ids.data())
                    : qf_encoder_generate_repairs(c.enc, 0, r, out_data + (size_t)*n * out_stride, out_stride,
                                                  lens.data(), co, ids.data());
    if (s == QF_ENOTREADY) return QF_OK;  // window not full: generate_repair_packet -> None
    if (s != QF_OK) return s;
    const uint32_t cb = c.coeff_bytes();
    if (out_coeffs && coeff_stride != cb) {
        // generate_repairs packs the coefficient blocks cb bytes apart: spread them
        for (uint32_t q = r; q-- > 1;)
            memmove(out_coeffs + (size_t)(*n + q) * coeff_stride, out_coeffs + (size_t)*n * coeff_stride + (size_t)q * cb,
                    cb);
    }
    for (uint32_t q = 0; q < r; ++q) {
        qf_packet_desc& d = desc[*n + q];
        d.id = ids[q];
        d.len = lens[q];
        d.coeff_len = cb;
        d.is_systematic = 0;
        d.reserved = 0;
    }
    *n += r;
    return QF_OK;
}

int drain_decoded(Codec& c, uint8_t* out_data, uint32_t out_stride, qf_packet_desc* desc,
                  uint32_t out_cap, uint32_t* n) {
    if (out_cap - *n < c.k) return QF_ETOOSMALL;
    std::vector<uint32_t> lens(c.k);
    std::vector<uint64_t> ids(c.k);
    uint32_t cnt = 0;
    int s = c.dec16 ? qf_decoder16_get_decoded_packets(c.dec16, out_data + (size_t)*n * out_stride, out_stride,
                                                       lens.data(), ids.data(), &cnt)
                    : qf_decoder_get_decoded_packets(c.dec, out_data + (size_t)*n * out_stride, out_stride, lens.data(),
                                                     ids.data(), &cnt);
    if (s != QF_OK) return s;
    for (uint32_t q = 0; q < cnt; ++q) {
        qf_packet_desc& d = desc[*n + q];
        d.id = ids[q];
        d.len = lens[q];
        d.coeff_len = 0;
        d.is_systematic = 1;
        d.reserved = 0;
    }
    *n += cnt;
    return QF_OK;
}

// DecoderVariant::add_packet + the was/now-decoded edge of on_receive
int receive_into(Codec& c, uint64_t id, int sys, const uint8_t* data, uint32_t len, const uint8_t* coeffs,
                 uint32_t coeff_len, uint8_t* out_data, uint32_t out_stride, qf_packet_desc* desc,
                 uint32_t out_cap, uint32_t* n) {
    if (c.k == 0 || !(c.dec || c.dec16)) {
        // Zero mode (decoder.rs:679: num_rows >= k) or no codec for the configuration
        if (!sys && !coeffs) return QF_EINVAL;
        return QF_OK;
    }
    const bool was = c.decoded;
    int s = c.dec16 ? qf_decoder16_add_packet(c.dec16, id, sys, data, len, coeffs, coeff_len)
                    : qf_decoder_add_packet(c.dec, id, sys, data, len, coeffs, coeff_len);
    if (s < 0) return s;
    c.decoded = s == 1;
    if (!was && c.decoded) return drain_decoded(c, out_data, out_stride, desc, out_cap, n);
    return QF_OK;
}

// qf_adaptive_on_send's argument checks (no state changes): *need = the
// packets the call may emit
int send_check(const qf_adaptive* a, uint32_t len, uint32_t out_stride, const uint8_t* out_coeffs,
               uint32_t coeff_stride, uint32_t* need) {
    if (len > a->cfg.max_len || out_stride < len) return QF_EINVAL;
    const bool fade_repairs = a->has_fade && a->transition_left > kFade / 2;
    *need = 1 + (a->cur.has_enc() ? a->cur.n - a->cur.k : 0) +
            (fade_repairs && a->fade.has_enc() ? a->fade.n - a->fade.k : 0);
    // repairs are window[0].len <= max_len bytes long: check the stride before
    // the windows advance, so a failing call leaves no state behind
    if (*need > 1 && out_stride < a->cfg.max_len) return QF_ETOOSMALL;
    if (out_coeffs) {
        uint32_t cmax = a->cur.has_enc() ? a->cur.coeff_bytes() : 0;
        if (fade_repairs && a->fade.has_enc() && a->fade.coeff_bytes() > cmax) cmax = a->fade.coeff_bytes();
        if (coeff_stride < cmax) return QF_ETOOSMALL;
    }
    return QF_OK;
}

void put_systematic(uint64_t id, const uint8_t* data, uint32_t len, uint8_t* out, qf_packet_desc* d) {
    if (len) memcpy(out, data, len);
    d->id = id;
    d->len = len;
    d->coeff_len = 0;
    d->is_systematic = 1;
    d->reserved = 0;
}

// adaptive.rs:537-543
void finish_send(qf_adaptive* a) {
    if (a->transition_left > 0) {
        a->transition_left--;
        if (a->transition_left == kFade / 2) {
            a->fade.release();
            a->has_fade = false;
        }
    }
}

}  // namespace

extern "C" {

void qf_fec_config_default(qf_fec_config* c) {
    if (!c) return;
    memset(c, 0, sizeof(*c));
    c->lambda = 0.1f;
    c->burst_window = 20;
    c->hysteresis = 0.02f;
    c->kp = 1.2f;
    c->ki = 0.5f;
    c->kd = 0.1f;
    c->initial_mode = QF_MODE_ZERO;
    c->kalman_enabled = 0;
    c->kalman_q = 0.001f;
    c->kalman_r = 0.01f;
    const uint32_t w[6] = {0, 16, 64, 128, 512, 1024};
    memcpy(c->window_sizes, w, sizeof(w));
    c->max_len = 1500;
}

int qf_fec_config_validate(const qf_fec_config* c) {
    if (!c) return QF_EINVAL;
    if (!(c->lambda >= 0.0f && c->lambda <= 1.0f)) return QF_EINVAL;
    if (c->burst_window == 0) return QF_EINVAL;
    if (!(c->hysteresis >= 0.0f && c->hysteresis < 1.0f)) return QF_EINVAL;
    if (c->kalman_enabled && (c->kalman_q <= 0.0f || c->kalman_r <= 0.0f)) return QF_EINVAL;
    if (!mode_ok(c->initial_mode)) return QF_EINVAL;
    return QF_OK;
}

int qf_mode_params_for(int32_t mode, uint32_t window, uint32_t* k, uint32_t* n) {
    if (!mode_ok(mode) || !k || !n) return QF_EINVAL;
    params_for(mode, window, k, n);
    return QF_OK;
}

int qf_mode_window_range(int32_t mode, uint32_t* lo, uint32_t* hi) {
    if (!mode_ok(mode) || !lo || !hi) return QF_EINVAL;
    *lo = kRangeLo[mode];
    *hi = kRangeHi[mode];
    return QF_OK;
}

float qf_mode_overhead_ratio(int32_t mode) { return mode_ok(mode) ? kRatio[mode] : 0.0f; }

int qf_adaptive_new_at(qf_ctx* ctx, const qf_fec_config* cfg, double now_s, qf_adaptive** out) {
    if (!cfg || !out) return QF_EINVAL;
    *out = nullptr;
    if (!mode_ok(cfg->initial_mode) || cfg->burst_window == 0 || cfg->max_len == 0) return QF_EINVAL;
    qf_adaptive* a = new qf_adaptive();
    a->ctx = ctx;
    a->cfg = *cfg;
    a->est.lambda = cfg->lambda;
    a->est.capacity = cfg->burst_window;
    a->est.use_kalman = cfg->kalman_enabled != 0;
    a->est.kf.q = cfg->kalman_q;
    a->est.kf.r = cfg->kalman_r;
    memcpy(a->mgr.windows, cfg->window_sizes, sizeof(a->mgr.windows));
    a->mgr.mode = cfg->initial_mode;
    a->mgr.window = a->mgr.windows[cfg->initial_mode];
    a->mgr.hysteresis = cfg->hysteresis;
    a->mgr.last_change = now_s;
    a->mgr.pid.kp = cfg->kp;
    a->mgr.pid.ki = cfg->ki;
    a->mgr.pid.kd = cfg->kd;
    a->mgr.pid.last_time = now_s;
    uint32_t k, n;
    params_for(a->mgr.mode, a->mgr.window, &k, &n);
    int s = make_codec(a, a->mgr.mode, k, n, &a->cur);
    if (s != QF_OK) {
        delete a;
        return s;
    }
    *out = a;
    return QF_OK;
}

int qf_adaptive_new(qf_ctx* ctx, const qf_fec_config* cfg, qf_adaptive** out) {
    return qf_adaptive_new_at(ctx, cfg, monotonic_s(), out);
}

int qf_adaptive_free(qf_adaptive* a) {
    if (!a) return QF_OK;
    a->cur.release();
    a->fade.release();
    delete a;
    return QF_OK;
}

int qf_adaptive_state(const qf_adaptive* a, int32_t* mode, uint32_t* window, uint32_t* k, uint32_t* n,
                      int32_t* transitioning, uint32_t* transition_left, float* estimated_loss) {
    if (!a) return QF_EINVAL;
    if (mode) *mode = a->mgr.mode;
    if (window) *window = a->mgr.window;
    if (k) *k = a->cur.k;
    if (n) *n = a->cur.n;
    if (transitioning) *transitioning = a->transition_left > 0;
    if (transition_left) *transition_left = a->transition_left;
    if (estimated_loss) *estimated_loss = a->est.estimate();
    return QF_OK;
}

uint32_t qf_adaptive_max_send_packets(const qf_adaptive* a) {
    if (!a) return 0;
    uint32_t m = 1;
    if (a->cur.has_enc()) m += a->cur.n - a->cur.k;
    if (a->has_fade && a->fade.has_enc()) m += a->fade.n - a->fade.k;
    return m;
}

// the need on_receive checks against out_cap (both decoders of a cross-fade)
uint32_t qf_adaptive_max_receive_packets(const qf_adaptive* a) {
    if (!a) return 0;
    return a->cur.k + (a->has_fade ? a->fade.k : 0);
}

uint32_t qf_adaptive_max_coeff_bytes(const qf_adaptive* a) {
    if (!a) return 0;
    uint32_t c = a->cur.has_enc() ? a->cur.coeff_bytes() : 0;
    if (a->has_fade && a->fade.has_enc() && a->fade.coeff_bytes() > c) c = a->fade.coeff_bytes();
    return c;
}

int qf_adaptive_on_send(qf_adaptive* a, uint64_t id, const uint8_t* data, uint32_t len, uint8_t* out_data,
                        uint32_t out_stride, uint8_t* out_coeffs, uint32_t coeff_stride, qf_packet_desc* out_desc,
                        uint32_t out_cap, uint32_t* n_out) {
    if (!a || !n_out || !out_data || !out_desc || (len && !data)) return QF_EINVAL;
    *n_out = 0;
    uint32_t need = 0;
    int s = send_check(a, len, out_stride, out_coeffs, coeff_stride, &need);
    if (s != QF_OK) return s;
    if (need > out_cap) return QF_ETOOSMALL;
    const bool fade_repairs = a->has_fade && a->transition_left > kFade / 2;
    // adaptive.rs:520-526: both encoders take a copy; the systematic packet is sent
    if (a->has_fade && (s = add_source(a->fade, id, data, len)) != QF_OK) return s;
    if ((s = add_source(a->cur, id, data, len)) != QF_OK) return s;
    uint32_t n = 0;
    put_systematic(id, data, len, out_data, out_desc);
    n = 1;
    if (fade_repairs && (s = emit_repairs(a->fade, out_data, out_stride, out_coeffs, coeff_stride, out_desc, &n)) != QF_OK)
        return s;
    if ((s = emit_repairs(a->cur, out_data, out_stride, out_coeffs, coeff_stride, out_desc, &n)) != QF_OK) return s;
    finish_send(a);
    *n_out = n;
    return a->cur.status;  // QF_ERANGE: the field has no code for this configuration
}

int qf_adaptive_on_send_batch(qf_adaptive* const* conns, uint32_t M, const uint64_t* ids, const uint8_t* const* data,
                              const uint32_t* lens, uint8_t* out_data, uint32_t out_stride, uint8_t* out_coeffs,
                              uint32_t coeff_stride, qf_packet_desc* out_desc, uint32_t out_cap, uint32_t* n_out,
                              int32_t* statuses) {
    if (M == 0) return QF_OK;
    if (!conns || !ids || !data || !lens || !out_data || !out_desc || !n_out) return QF_EINVAL;
    // every argument check before any state changes: a connection's need
    // does not grow from one on_send to the next (only report_loss starts a
    // cross-fade), so the current state bounds repeated connections too
    uint64_t total = 0;
    for (uint32_t m = 0; m < M; ++m) {
        if (!conns[m] || (lens[m] && !data[m])) return QF_EINVAL;
        uint32_t need = 0;
        int s = send_check(conns[m], lens[m], out_stride, out_coeffs, coeff_stride, &need);
        if (s != QF_OK) return s;
        total += need;
        n_out[m] = 0;
        if (statuses) statuses[m] = QF_OK;
    }
    if (total > out_cap) return QF_ETOOSMALL;
    uint32_t pos = 0;
    std::vector<qf::EncSend> batch;
    std::vector<uint32_t> batch_m, predicted;
    // packets of a steady connection already in this segment's batch: a
    // connection may repeat (a burst), its windows then overlap and go to the
    // device in the same launch (encoders_send_batch)
    std::unordered_map<const qf_adaptive*, uint32_t> queued;
    queued.reserve(M);
    for (uint32_t m0 = 0; m0 < M;) {
        // a segment: normally the whole call (a connection of another
        // context takes the per-packet path inline, as a cross-fade does)
        batch.clear();
        batch_m.clear();
        predicted.clear();
        queued.clear();
        qf_ctx* ctx = nullptr;
        uint32_t m = m0;
        for (; m < M; ++m) {
            qf_adaptive* a = conns[m];
            const bool steady = a->ctx && !a->has_fade && a->cur.enc && (!ctx || a->ctx == ctx);
            if (!steady && queued.count(a)) break;   // its queued packets go first
            if (!steady) {  // cross-fade, GF(2^16), Zero mode, controller only: one on_send
                uint32_t n = 0;
                int s = qf_adaptive_on_send(a, ids[m], data[m], lens[m], out_data + (size_t)pos * out_stride,
                                            out_stride, out_coeffs ? out_coeffs + (size_t)pos * coeff_stride : nullptr,
                                            coeff_stride, out_desc + pos, out_cap - pos, &n);
                if (s < 0 && s != QF_ERANGE) return s;
                if (statuses) statuses[m] = s;
                n_out[m] = n;
                pos += n;
                continue;
            }
            ctx = a->ctx;
            const Codec& c = a->cur;
            uint32_t& q = queued[a];
            const uint32_t cnt = std::min<uint32_t>((uint32_t)qf_encoder_window_len(c.enc) + q++, c.k);
            const uint32_t n_rep = (cnt + 1 >= c.k && c.n > c.k) ? c.n - c.k : 0;
            put_systematic(ids[m], data[m], lens[m], out_data + (size_t)pos * out_stride, out_desc + pos);
            qf::EncSend x{};
            x.e = c.enc;
            x.id = ids[m];
            x.data = data[m];
            x.len = lens[m];
            x.rep_data = out_data + (size_t)(pos + 1) * out_stride;
            x.rep_stride = out_stride;
            x.rep_coeffs = out_coeffs ? out_coeffs + (size_t)(pos + 1) * coeff_stride : nullptr;
            x.coeff_stride = coeff_stride;
            x.rep_desc = out_desc + pos + 1;
            batch.push_back(x);
            batch_m.push_back(m);
            predicted.push_back(n_rep);
            n_out[m] = 1 + n_rep;
            pos += 1 + n_rep;
        }
        if (batch.size() == 1) {
            // one steady connection: the per-packet path (no staging table,
            // no scatter launch); its rows were placed above, rerun in place
            const uint32_t mm = batch_m[0];
            const uint32_t p0 = (uint32_t)(batch[0].rep_desc - out_desc) - 1;
            uint32_t n = 0;
            int s = qf_adaptive_on_send(conns[mm], ids[mm], data[mm], lens[mm], out_data + (size_t)p0 * out_stride,
                                        out_stride, out_coeffs ? out_coeffs + (size_t)p0 * coeff_stride : nullptr,
                                        coeff_stride, out_desc + p0, out_cap - p0, &n);
            if (s < 0 && s != QF_ERANGE) return s;
            if (n != predicted[0] + 1) return qf::device_fail(__FILE__, __LINE__, hipErrorIllegalState);  // internal inconsistency
            if (statuses) statuses[mm] = s;
        } else if (!batch.empty()) {
            int s = qf::encoders_send_batch(ctx, batch.data(), (uint32_t)batch.size());
            if (s != QF_OK) return s;
            for (size_t b = 0; b < batch.size(); ++b) {
                if (batch[b].n_rep != predicted[b]) return qf::device_fail(__FILE__, __LINE__, hipErrorIllegalState);  // internal inconsistency
                finish_send(conns[batch_m[b]]);
            }
        }
        m0 = m;
    }
    return QF_OK;
}

int qf_adaptive_on_receive(qf_adaptive* a, uint64_t id, int is_systematic, const uint8_t* data, uint32_t len,
                           const uint8_t* coeffs, uint32_t coeff_len, uint8_t* out_data, uint32_t out_stride,
                           qf_packet_desc* out_desc, uint32_t out_cap, uint32_t* n_out) {
    if (!a || !n_out || (len && !data)) return QF_EINVAL;
    *n_out = 0;
    uint32_t need = a->cur.k + (a->has_fade ? a->fade.k : 0);
    if (need && (!out_data || !out_desc || out_cap < need || out_stride < a->cfg.max_len)) return QF_ETOOSMALL;
    const bool to_fade = a->has_fade && a->transition_left > kFade / 2;
    uint32_t n = 0;
    int s = receive_into(a->cur, id, is_systematic, data, len, coeffs, coeff_len, out_data, out_stride, out_desc,
                         out_cap, &n);
    if (s != QF_OK) return s;
    if (to_fade) {
        s = receive_into(a->fade, id, is_systematic, data, len, coeffs, coeff_len, out_data, out_stride, out_desc,
                         out_cap, &n);
        if (s != QF_OK) return s;
    }
    *n_out = n;
    return QF_OK;
}

int qf_adaptive_on_receive_batch(qf_adaptive* const* conns, uint32_t M, const uint64_t* ids,
                                 const int32_t* is_systematic, const uint8_t* const* data, const uint32_t* lens,
                                 const uint8_t* const* coeffs, const uint32_t* coeff_lens, uint8_t* out_data,
                                 uint32_t out_stride, qf_packet_desc* out_desc, uint32_t out_cap, uint32_t* n_out,
                                 int32_t* statuses) {
    if (M == 0) return QF_OK;
    if (!conns || !ids || !is_systematic || !data || !lens || !n_out) return QF_EINVAL;
    // every argument check before any state changes (as the send batch): a
    // connection's need (the k of its decoders) does not change on receive
    uint64_t total = 0;
    for (uint32_t m = 0; m < M; ++m) {
        const qf_adaptive* a = conns[m];
        if (!a || (lens[m] && !data[m])) return QF_EINVAL;
        const uint32_t need = a->cur.k + (a->has_fade ? a->fade.k : 0);
        if (need && (!out_data || !out_desc || out_stride < a->cfg.max_len)) return QF_ETOOSMALL;
        total += need;
        n_out[m] = 0;
        if (statuses) statuses[m] = QF_OK;
    }
    if (total > out_cap) return QF_ETOOSMALL;
    uint32_t pos = 0;
    std::vector<qf::DecAdd> batch;
    std::vector<uint32_t> batch_m;
    std::vector<uint8_t> was;
    std::unordered_set<const qf_adaptive*> seen;
    seen.reserve(M);
    for (uint32_t m0 = 0; m0 < M;) {
        // a segment: each connection at most once (a repeat starts the next)
        batch.clear();
        batch_m.clear();
        was.clear();
        seen.clear();
        qf_ctx* ctx = nullptr;
        uint32_t m = m0;
        for (; m < M; ++m) {
            qf_adaptive* a = conns[m];
            if (!seen.insert(a).second) break;
            const bool to_fade = a->has_fade && a->transition_left > kFade / 2;
            if (a->ctx && a->cur.dec && !to_fade && a->cur.k > 0 && (!ctx || a->ctx == ctx)) {
                ctx = a->ctx;
                qf::DecAdd x{};
                x.d = a->cur.dec;
                x.id = ids[m];
                x.is_systematic = is_systematic[m];
                x.data = data[m];
                x.len = lens[m];
                x.coeffs = coeffs ? coeffs[m] : nullptr;
                x.coeff_len = coeff_lens ? coeff_lens[m] : 0;
                batch.push_back(x);
                batch_m.push_back(m);
                was.push_back(a->cur.decoded ? 1 : 0);
            }
        }
        if (batch.size() == 1) {   // one connection: the per-packet path (no staging, no scatter launch)
            batch.clear();
            batch_m.clear();
            was.clear();
        }
        if (!batch.empty()) {
            int s = qf::decoders_add_batch(ctx, batch.data(), (uint32_t)batch.size());
            if (s != QF_OK) return s;
        }
        // outputs in connection order: batched connections drain their decoders,
        // the others run the per-packet on_receive here
        for (uint32_t i = m0, b = 0; i < m; ++i) {
            qf_adaptive* a = conns[i];
            uint32_t n = 0;
            int s;
            if (b < batch_m.size() && batch_m[b] == i) {
                const qf::DecAdd& x = batch[b];
                Codec& c = a->cur;
                s = x.result < 0 ? x.result : QF_OK;
                if (s == QF_OK) {
                    c.decoded = x.result == 1;
                    if (!was[b] && c.decoded)
                        s = drain_decoded(c, out_data + (size_t)pos * out_stride, out_stride, out_desc + pos,
                                          out_cap - pos, &n);
                    // drain_decoded writes from row 0 of the slice it is given
                    // (its *n starts at 0)
                }
                ++b;
            } else {
                s = qf_adaptive_on_receive(a, ids[i], is_systematic[i], data[i], lens[i], coeffs ? coeffs[i] : nullptr,
                                           coeff_lens ? coeff_lens[i] : 0, out_data ? out_data + (size_t)pos * out_stride : nullptr,
                                           out_stride, out_desc ? out_desc + pos : nullptr, out_cap - pos, &n);
            }
            if (s < 0) {
                if (statuses) statuses[i] = s;
                n = 0;
            }
            n_out[i] = n;
            pos += n;
        }
        m0 = m;
    }
    return QF_OK;
}

int qf_adaptive_report_loss_at(qf_adaptive* a, uint32_t lost, uint32_t total, double now_s) {
    if (!a || lost > total) return QF_EINVAL;
    a->est.report(lost, total);
    const float e = a->est.estimate();
    int32_t pm = 0;
    uint32_t pw = 0;
    const bool fade = a->mgr.update(e, now_s, &pm, &pw);
    uint32_t k, n;
    params_for(a->mgr.mode, a->mgr.window, &k, &n);
    Codec fresh;
    int s = make_codec(a, a->mgr.mode, k, n, &fresh);
    if (s != QF_OK) return s;
    if (fade) {
        // adaptive.rs:612-624: keep the old configuration for the cross-fade
        a->fade.release();
        a->fade = a->cur;
        a->has_fade = true;
        a->transition_left = kFade;
    } else {
        a->cur.release();  // adaptive.rs:626-629
    }
    a->cur = fresh;
    return QF_OK;
}

int qf_adaptive_report_loss(qf_adaptive* a, uint32_t lost, uint32_t total) {
    return qf_adaptive_report_loss_at(a, lost, total, monotonic_s());
}

}  // extern "C"
