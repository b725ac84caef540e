// Native driver of the reference's benches/fec_modes.rs through the C-ABI
// (no Python, no torch: links libqf_fec_rocm.so).  Three parts, one JSON
// object on stdout:
//
//  send      AdaptiveFec::on_send (adaptive.rs:519-562) of a 1,024-byte 0xAB
//            packet per mode (fec_modes.rs:9-45), window full, so every call
//            slides the window and emits n - k repairs: microseconds per call.
//  receive   AdaptiveFec::on_receive (adaptive.rs:566-599) per packet in the
//            same modes: a generation of k sources with 20 % of them lost,
//            then the window's repairs until it decodes; microseconds per
//            call, and the call that completes the generation (the decode)
//            on its own.  A loss report between generations rebuilds the
//            codecs (adaptive.rs:602-630), outside the timed calls.
//  batch1    ONE connection's packets through qf_adaptive_on_send_batch, the
//            connection repeated B times in the call (B = 1, 16, 256; Normal
//            mode, 1,200-B packets): packets per second for one connection.
//
//   make -C tools/send_batch      (-> tools/send_batch/build/bench_on_send)
//   tools/send_batch/build/bench_on_send [calls]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "qf_fec.h"

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define QF(call)                                                                                      \
    do {                                                                                              \
        int s_ = (call);                                                                              \
        if (s_ != QF_OK) {                                                                            \
            fprintf(stderr, "FAIL %s:%d %s -> %s\n", __FILE__, __LINE__, #call, qf_strerror(s_));    \
            exit(1);                                                                                  \
        }                                                                                             \
    } while (0)

struct Stats {
    double mean, median, p99;
};

static Stats stats(std::vector<double> t) {
    Stats s{0, 0, 0};
    if (t.empty()) return s;
    std::sort(t.begin(), t.end());
    double sum = 0;
    for (double v : t) sum += v;
    s.mean = sum / t.size();
    s.median = t[t.size() / 2];
    s.p99 = t[(t.size() * 99) / 100 < t.size() ? (t.size() * 99) / 100 : t.size() - 1];
    return s;
}

static const char* kNames[] = {"Zero", "Light", "Normal", "Medium", "Strong", "Extreme"};

static void send_part(qf_ctx* ctx, int calls) {
    const uint32_t len = 1024;
    std::vector<uint8_t> payload(len, 0xAB);  // fec_modes.rs:9-12
    printf("\"send\": {\"len\": %u, \"calls\": %d, \"modes\": {", len, calls);
    bool first = true;
    for (int32_t mode : {QF_MODE_LIGHT, QF_MODE_NORMAL, QF_MODE_MEDIUM, QF_MODE_STRONG, QF_MODE_EXTREME}) {
        qf_fec_config cfg;
        qf_fec_config_default(&cfg);
        cfg.initial_mode = mode;
        cfg.max_len = 2048;
        qf_adaptive* a = nullptr;
        QF(qf_adaptive_new_at(ctx, &cfg, 0.0, &a));
        uint32_t k = 0, n = 0;
        qf_adaptive_state(a, nullptr, nullptr, &k, &n, nullptr, nullptr, nullptr);
        const uint32_t cap = qf_adaptive_max_send_packets(a);
        const uint32_t stride = 2048, cstride = std::max<uint32_t>(qf_adaptive_max_coeff_bytes(a), 1);
        std::vector<uint8_t> out((size_t)cap * stride), coeffs((size_t)cap * cstride);
        std::vector<qf_packet_desc> desc(cap);
        uint64_t id = 0;
        uint32_t n_out = 0;
        int st = QF_OK;
        for (uint32_t i = 0; i < k + 8; ++i)   // window full: the bench's steady state
            st = qf_adaptive_on_send(a, id++, payload.data(), len, out.data(), stride, coeffs.data(), cstride,
                                     desc.data(), cap, &n_out);
        std::vector<double> t(calls);
        uint64_t repairs = 0;
        for (int c = 0; c < calls; ++c) {
            const double t0 = now_us();
            st = qf_adaptive_on_send(a, id++, payload.data(), len, out.data(), stride, coeffs.data(), cstride,
                                     desc.data(), cap, &n_out);
            t[c] = now_us() - t0;
            repairs += n_out ? n_out - 1 : 0;
        }
        const Stats s = stats(t);
        printf("%s\"%s\": {\"k\": %u, \"n\": %u, \"status\": %d, \"us_mean\": %.2f, \"us_median\": %.2f, "
               "\"us_p99\": %.2f, \"repairs_per_call\": %.2f, \"repair_mib_per_s\": %.1f}",
               first ? "" : ", ", kNames[mode], k, n, st, s.mean, s.median, s.p99, (double)repairs / calls,
               (double)repairs * len / (s.mean * calls / 1e6) / (1 << 20));
        first = false;
        qf_adaptive_free(a);
    }
    printf("}}");
}

static void receive_part(qf_ctx* ctx, int gens) {
    const uint32_t len = 1024;
    printf("\"receive\": {\"len\": %u, \"generations\": %d, \"loss\": 0.2, \"modes\": {", len, gens);
    bool first = true;
    for (int32_t mode : {QF_MODE_LIGHT, QF_MODE_NORMAL, QF_MODE_MEDIUM, QF_MODE_EXTREME}) {
        qf_fec_config cfg;
        qf_fec_config_default(&cfg);
        cfg.initial_mode = mode;
        cfg.max_len = 2048;
        qf_adaptive *snd = nullptr, *rcv = nullptr;
        QF(qf_adaptive_new_at(ctx, &cfg, 0.0, &snd));
        QF(qf_adaptive_new_at(ctx, &cfg, 0.0, &rcv));
        uint32_t k = 0, n = 0;
        qf_adaptive_state(snd, nullptr, nullptr, &k, &n, nullptr, nullptr, nullptr);
        const uint32_t r = n - k, e = std::min<uint32_t>(r, std::max<uint32_t>(1, (k + 2) / 5));
        const uint32_t scap = qf_adaptive_max_send_packets(snd), stride = 2048;
        const uint32_t cstride = std::max<uint32_t>(qf_adaptive_max_coeff_bytes(snd), 1);
        std::vector<uint8_t> out((size_t)scap * stride), coeffs((size_t)scap * cstride), src((size_t)k * len);
        std::vector<uint8_t> rep((size_t)r * len), rco((size_t)r * cstride);
        std::vector<qf_packet_desc> desc(scap);
        const uint32_t rcap = std::max<uint32_t>(qf_adaptive_max_receive_packets(rcv), 1);
        std::vector<uint8_t> rout((size_t)rcap * stride);
        std::vector<qf_packet_desc> rdesc(rcap);
        std::vector<double> per_packet, decode_call;
        int ok_gens = 0;
        uint64_t seed = 0x51464543u + mode;
        for (int g = 0; g < gens; ++g) {
            for (auto& b : src) b = (uint8_t)((seed = seed * 6364136223846793005ull + 1) >> 56);
            uint32_t n_out = 0;
            for (uint32_t i = 0; i < k; ++i) {
                QF(qf_adaptive_on_send(snd, i, src.data() + (size_t)i * len, len, out.data(), stride, coeffs.data(),
                                       cstride, desc.data(), scap, &n_out));
                for (uint32_t j = 0; j + 1 < n_out; ++j) {
                    memcpy(rep.data() + (size_t)j * len, out.data() + (size_t)(1 + j) * stride, len);
                    memcpy(rco.data() + (size_t)j * cstride, coeffs.data() + (size_t)(1 + j) * cstride,
                           desc[1 + j].coeff_len);
                }
            }
            const uint32_t cl = desc[1].coeff_len;
            uint32_t got = 0, m = 0;
            for (uint32_t i = 0; i < k && got < k; ++i) {
                if ((i * 7 + g) % k < e) continue;   // e of the k sources lost
                const double t0 = now_us();
                QF(qf_adaptive_on_receive(rcv, i, 1, src.data() + (size_t)i * len, len, nullptr, 0, rout.data(),
                                          stride, rdesc.data(), rcap, &m));
                const double dt = now_us() - t0;
                per_packet.push_back(dt);
                if (m) decode_call.push_back(dt);
                got += m;
            }
            for (uint32_t j = 0; j < r && got < k; ++j) {
                const double t0 = now_us();
                QF(qf_adaptive_on_receive(rcv, k + j, 0, rep.data() + (size_t)j * len, len,
                                          rco.data() + (size_t)j * cstride, cl, rout.data(), stride, rdesc.data(),
                                          rcap, &m));
                const double dt = now_us() - t0;
                per_packet.push_back(dt);
                if (m) decode_call.push_back(dt);
                got += m;
            }
            ok_gens += got == k;
            QF(qf_adaptive_report_loss_at(snd, 0, 100, 0.0));
            QF(qf_adaptive_report_loss_at(rcv, 0, 100, 0.0));
        }
        const Stats s = stats(per_packet), d = stats(decode_call);
        printf("%s\"%s\": {\"k\": %u, \"n\": %u, \"lost\": %u, \"recovered_generations\": %d, \"calls\": %zu, "
               "\"us_mean\": %.2f, \"us_median\": %.2f, \"us_p99\": %.2f, \"decode_call_us_median\": %.2f}",
               first ? "" : ", ", kNames[mode], k, n, e, ok_gens, per_packet.size(), s.mean, s.median, s.p99,
               d.median);
        first = false;
        qf_adaptive_free(snd);
        qf_adaptive_free(rcv);
    }
    printf("}}");
}

static void batch_one_connection(qf_ctx* ctx, int rounds) {
    const uint32_t len = 1200;
    printf("\"batch1\": {\"mode\": \"Normal\", \"len\": %u, \"per_call\": {", len);
    bool first = true;
    for (uint32_t B : {1u, 16u, 256u}) {
        qf_fec_config cfg;
        qf_fec_config_default(&cfg);
        cfg.initial_mode = QF_MODE_NORMAL;
        cfg.max_len = len;
        qf_adaptive* a = nullptr;
        QF(qf_adaptive_new_at(ctx, &cfg, 0.0, &a));
        const uint32_t per = qf_adaptive_max_send_packets(a), cap = per * B;
        const uint32_t cstride = std::max<uint32_t>(qf_adaptive_max_coeff_bytes(a), 1);
        std::vector<uint8_t> out((size_t)cap * len), coeffs((size_t)cap * cstride), pk((size_t)B * len, 0xAB);
        std::vector<qf_packet_desc> desc(cap);
        std::vector<qf_adaptive*> conns(B, a);
        std::vector<uint64_t> ids(B);
        std::vector<const uint8_t*> data(B);
        std::vector<uint32_t> lens(B, len), n_out(B);
        std::vector<int32_t> st(B);
        uint64_t id = 0;
        auto call = [&]() {
            for (uint32_t b = 0; b < B; ++b) ids[b] = id++, data[b] = pk.data() + (size_t)b * len;
            QF(qf_adaptive_on_send_batch(conns.data(), B, ids.data(), data.data(), lens.data(), out.data(), len,
                                         coeffs.data(), cstride, desc.data(), cap, n_out.data(), st.data()));
        };
        while (id < 2 * 64 + 8) call();   // window full
        const int calls = std::max(4, rounds / (int)B);
        uint64_t packets = 0, repairs = 0;
        const double t0 = now_us();
        for (int c = 0; c < calls; ++c) {
            call();
            packets += B;
            for (uint32_t b = 0; b < B; ++b) repairs += n_out[b] ? n_out[b] - 1 : 0;
        }
        const double us = now_us() - t0;
        printf("%s\"%u\": {\"calls\": %d, \"us_per_call\": %.2f, \"us_per_packet\": %.3f, \"packets_per_s\": %.0f, "
               "\"repairs_per_packet\": %.2f}",
               first ? "" : ", ", B, calls, us / calls, us / packets, packets / (us / 1e6), (double)repairs / packets);
        first = false;
        qf_adaptive_free(a);
    }
    printf("}}");
}

int main(int argc, char** argv) {
    const int calls = argc > 1 ? atoi(argv[1]) : 300;
    qf_ctx* ctx = nullptr;
    if (qf_ctx_create(0, nullptr, &ctx) != QF_OK) {
        fprintf(stderr, "qf_ctx_create failed\n");
        return 1;
    }
    printf("{\"tool\": \"tools/bench_on_send.cpp\", ");
    send_part(ctx, calls);
    printf(", ");
    receive_part(ctx, 8);
    printf(", ");
    batch_one_connection(ctx, 4096);
    printf("}\n");
    qf_ctx_destroy(ctx);
    return 0;
}
