// scripts/strip_probe.cpp — VERDICT r4 item 5 probe: strip the timestamps of query_range bodies while
// staging them (what the device packer would need to send fewer bytes over PCIe) vs the plain
// staging memcpy, one thread.  g++ -O3 -march=native scripts/strip_probe.cpp -o /tmp/strip && /tmp/strip
// timestamp-strip staging filter vs memcpy, one thread, on query_range-shaped JSON
#include <chrono>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>
int main() {
    std::mt19937_64 g(1);
    std::gamma_distribution<double> ga(2, 0.05);
    std::string body = "{\"status\":\"success\",\"data\":{\"resultType\":\"matrix\",\"result\":[{\"metric\":{},\"values\":[";
    char buf[64];
    for (int i = 0; i < 10080 * 30; ++i) {
        snprintf(buf, 64, "[%d.25,\"%.17g\"]%s", 1700000000 + 60 * i, ga(g), i + 1 < 10080 * 30 ? "," : "");
        body += buf;
    }
    body += "]}]}}";
    std::vector<char> dst(body.size());
    const int R = 20;
    auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < R; ++r) memcpy(dst.data(), body.data(), body.size());
    auto t1 = std::chrono::steady_clock::now();
    size_t out = 0;
    for (int r = 0; r < R; ++r) {
        const char* p = body.data();
        const char* e = p + body.size();
        char* o = dst.data();
        // keep ["value"] of each element: skip '[' + timestamp + ','
        const char* v = (const char*)memmem(p, e - p, "\"values\":[", 10) + 10;
        memcpy(o, p, v - p); o += v - p; p = v;
        while (p < e && *p == '[') {
            const char* c = (const char*)memchr(p, ',', e - p);
            const char* q = (const char*)memchr(c + 2, '"', e - c - 2);
            memcpy(o, c + 1, q - c); o += q - c;  // "value"
            p = q + 2;  // past '"' and ']'
            if (p < e && *p == ',') { *o++ = ','; ++p; }
        }
        memcpy(o, p, e - p); o += e - p;
        out = o - dst.data();
    }
    auto t2 = std::chrono::steady_clock::now();
    double gb = (double)body.size() * R / 1e9;
    printf("body %.1f MB -> %.1f MB (%.0f%%): memcpy %.1f GB/s, strip %.1f GB/s per thread\n", body.size() / 1e6,
           out / 1e6, 100.0 * out / body.size(), gb / std::chrono::duration<double>(t1 - t0).count(),
           gb / std::chrono::duration<double>(t2 - t1).count());
}
