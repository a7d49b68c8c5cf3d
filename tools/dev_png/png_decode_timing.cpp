#include <chrono>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>
namespace ik { int decode_png(const uint8_t*, size_t, uint32_t&, uint32_t&, uint32_t&, std::vector<uint8_t>&); }
int main() {
    FILE* f = fopen("s.png", "rb"); std::vector<uint8_t> b(1 << 27); size_t n = fread(b.data(), 1, b.size(), f); fclose(f);
    std::vector<uint8_t> raw(4096ull * 4096 * 4); f = fopen("s.raw", "rb"); fread(raw.data(), 1, raw.size(), f); fclose(f);
    for (int it = 0; it < 3; ++it) {
        uint32_t w, h, c; static std::vector<uint8_t> px;
        auto t0 = std::chrono::steady_clock::now();
        int rc = ik::decode_png(b.data(), n, w, h, c, px);
        double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        printf("rc=%d %ux%ux%u %.1f ms equal=%d\n", rc, w, h, c, ms, px.size() == raw.size() && !memcmp(px.data(), raw.data(), raw.size()));
    }
}
