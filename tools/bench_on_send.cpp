// Native driver of the reference's benches/fec_modes.rs through the C-ABI:
// AdaptiveFec::on_send (adaptive.rs:519-562) of a 1,024-byte 0xAB packet per
// mode, window full, so every call slides the window and emits n - k repairs.
// Same work as tools/bench_fec_modes.py, without the Python mirror / ctypes
// in the timed loop.  Prints one JSON object.
//
//   g++ -O2 -std=c++17 -Iinclude tools/bench_on_send.cpp -Lquicfuscate_amd/lib -lqf_fec \
//       -Wl,-rpath,'$ORIGIN/../quicfuscate_amd/lib' -o tools/bench_on_send
//   tools/bench_on_send [calls]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "qf_fec.h"

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const int calls = argc > 1 ? atoi(argv[1]) : 300;
    const uint32_t len = 1024;
    qf_ctx* ctx = nullptr;
    if (qf_ctx_create(0, nullptr, &ctx) != QF_OK) {
        fprintf(stderr, "qf_ctx_create failed\n");
        return 1;
    }
    std::vector<uint8_t> payload(len, 0xAB);  // fec_modes.rs:9-12
    const char* names[] = {"Zero", "Light", "Normal", "Medium", "Strong", "Extreme"};
    printf("{\"tool\": \"tools/bench_on_send.cpp\", \"len\": %u, \"calls\": %d, \"modes\": {", len, calls);
    bool first = true;
    for (int32_t mode : {QF_MODE_LIGHT, QF_MODE_NORMAL, QF_MODE_MEDIUM, QF_MODE_STRONG, QF_MODE_EXTREME}) {
        qf_fec_config cfg;
        qf_fec_config_default(&cfg);
        cfg.initial_mode = mode;
        cfg.max_len = 2048;
        qf_adaptive* a = nullptr;
        if (qf_adaptive_new_at(ctx, &cfg, 0.0, &a) != QF_OK) {
            fprintf(stderr, "qf_adaptive_new failed for mode %d\n", mode);
            return 1;
        }
        uint32_t window = 0, k = 0, n = 0;
        qf_adaptive_state(a, nullptr, &window, &k, &n, nullptr, nullptr, nullptr);
        const uint32_t cap = qf_adaptive_max_send_packets(a);
        const uint32_t stride = 2048, cstride = 2 * std::max<uint32_t>(k, 1) + 16;
        std::vector<uint8_t> out((size_t)cap * stride), coeffs((size_t)cap * cstride);
        std::vector<qf_packet_desc> desc(cap);
        uint64_t id = 0;
        uint32_t n_out = 0;
        int st = QF_OK;
        // fill the window (the reference bench runs long enough to be in steady state)
        for (uint32_t i = 0; i < k + 8; ++i)
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
        std::sort(t.begin(), t.end());
        double sum = 0;
        for (double v : t) sum += v;
        printf("%s\"%s\": {\"k\": %u, \"n\": %u, \"status\": %d, \"us_mean\": %.2f, \"us_median\": %.2f, "
               "\"us_p99\": %.2f, \"repairs_per_call\": %.2f, \"repair_mib_per_s\": %.1f}",
               first ? "" : ", ", names[mode], k, n, st, sum / calls, t[calls / 2], t[(calls * 99) / 100],
               (double)repairs / calls, (double)repairs * len / (sum / 1e6) / (1 << 20));
        first = false;
        qf_adaptive_free(a);
    }
    printf("}}\n");
    qf_ctx_destroy(ctx);
    return 0;
}
