// scripts/strip_bench.cpp — the staging strip (krr_amd/csrc/krr_strip.h) against memcpy on
// config-1-shaped bodies, 1..T threads, ~1 GB per pass (out of cache), on the host it runs on.
// g++ -O3 -std=c++17 -pthread -Ikrr_amd/csrc [-DKRR_STRIP_MASKED_STORES=0] scripts/strip_bench.cpp -o strip_bench
#include "krr_strip.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <thread>
#include <vector>

int main(int argc, char** argv) {
    std::mt19937_64 g(1);
    std::gamma_distribution<double> ga(2, 0.05);
    std::string body = "{\"status\":\"success\",\"data\":{\"resultType\":\"matrix\",\"result\":[{\"metric\":{\"pod\":\"p\"},\"values\":[";
    char buf[64];
    for (int i = 0; i < 10080; ++i) {
        snprintf(buf, 64, "[%.1f,\"%.17g\"]%s", 1.7e9 + 60 * i, ga(g), i + 1 < 10080 ? "," : "");
        body += buf;
    }
    body += "]}]}}";
    const size_t NB = 2800;  // ~1 GB
    std::vector<char> src(body.size() * NB), dst(body.size() * NB + 64);
    for (size_t i = 0; i < NB; ++i) memcpy(src.data() + i * body.size(), body.data(), body.size());
    printf("strip supported: %d, masked stores: %d\n", (int)krr::strip::supported(), KRR_STRIP_MASKED_STORES);
    for (int T : {1, 4, 8, 12, 16}) {
        for (int mode = 0; mode < 3; ++mode) {  // memcpy, strip, strip into a per-thread 1-MB ring (no DRAM writes)
            double best = 1e9;
            for (int rep = 0; rep < 3; ++rep) {
                auto t0 = std::chrono::steady_clock::now();
                std::vector<std::thread> th;
                for (int t = 0; t < T; ++t)
                    th.emplace_back([&, t] {
                        std::vector<char> ring(mode == 2 ? body.size() + 64 : 0);
                        for (size_t i = t; i < NB; i += T) {
                            const char* s = src.data() + i * body.size();
                            char* o = mode == 2 ? ring.data() : dst.data() + i * body.size();
                            if (mode) krr::strip::strip_body(s, body.size(), o);
                            else memcpy(o, s, body.size());
                        }
                    });
                for (auto& x : th) x.join();
                best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
            }
            printf("%-9s T=%2d: %6.1f GB/s of JSON (%.2f per thread)\n", mode == 2 ? "strip-ring" : mode ? "strip" : "memcpy", T,
                   src.size() / best / 1e9, src.size() / best / 1e9 / T);
        }
    }
}
