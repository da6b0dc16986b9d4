// scripts/strip_prefetch_bench.cpp — the staging strip (krr_amd/csrc/krr_strip.h) over source
// bodies on 4-KiB pages (as Python bytes objects are: the bench's grouped bodies show no
// transparent huge pages) with software prefetch PF bytes ahead, T threads each stripping its
// own run of whole bodies, ~2 GB per pass.
// g++ -O3 -std=c++17 -pthread -Ikrr_amd/csrc scripts/strip_prefetch_bench.cpp -o strip_prefetch_bench
#include "krr_strip.h"

#include <sys/mman.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <cstdio>
#include <random>
#include <string>
#include <thread>
#include <vector>

template <int PF>
int64_t run(const char* s, int64_t n, char* o) {
    return krr::strip::strip_span_t<false, PF>(s, s + n, o, nullptr);
}

int main() {
    std::mt19937_64 g(1);
    std::gamma_distribution<double> ga(2, 0.05);
    std::string body;
    char buf[64];
    for (int i = 0; i < 10080; ++i) {
        snprintf(buf, 64, "[%.1f,\"%.17g\"]%s", 1.7e9 + 60 * i, ga(g), i + 1 < 10080 ? "," : "");
        body += buf;
    }
    const size_t NB = 6000;  // ~2 GB
    const size_t total = body.size() * NB;
    char* src = (char*)mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    char* dst = (char*)mmap(nullptr, total + 64, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    madvise(src, total, MADV_NOHUGEPAGE);
    madvise(dst, total + 64, MADV_HUGEPAGE);
    for (size_t i = 0; i < NB; ++i) memcpy(src + i * body.size(), body.data(), body.size());
    memset(dst, 0, total + 64);
    printf("strip supported: %d, %.2f GB of JSON on 4-KiB pages\n", (int)krr::strip::supported(), total / 1e9);
    using Fn = int64_t (*)(const char*, int64_t, char*);
    const std::pair<int, Fn> variants[] = {{0, run<0>}, {512, run<512>}, {1024, run<1024>}, {2048, run<2048>},
                                           {4096, run<4096>}};
    for (int T : {1, 8, 16}) {
        for (int round = 0; round < 2; ++round) {
            for (const auto& [pf, fn] : variants) {
                double best = 1e9;
                for (int rep = 0; rep < 3; ++rep) {
                    auto t0 = std::chrono::steady_clock::now();
                    std::vector<std::thread> th;
                    const size_t bs = body.size();
                    for (int t = 0; t < T; ++t)
                        th.emplace_back([&, t] {
                            for (size_t i = NB * t / T; i < NB * (t + 1) / T; ++i)
                                if (fn(src + i * bs, (int64_t)bs, dst + i * bs) < 0) abort();
                        });
                    for (auto& x : th) x.join();
                    best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
                }
                printf("T=%2d PF=%5d: %6.1f GB/s of JSON (%.2f per thread)\n", T, pf, total / best / 1e9,
                       total / best / 1e9 / T);
            }
        }
    }
}
