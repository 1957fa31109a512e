// ASan/UBSan fuzz of fa_bson_elements and fa_bson_walk (host only, no GPU):
//   g++ -std=c++17 -g -O1 -fsanitize=address,undefined -Iinclude tools/bson_fuzz.cpp \
//       fedlesscan_amd/csrc/bson_host.cpp -o tools/build/bson_fuzz && tools/build/bson_fuzz seed.bson
// Every truncation of the seed, then random 1-4 byte mutations; each parse walks
// nested documents/arrays recursively with fa_bson_elements and must agree
// with the one-call fa_bson_walk (same verdict, same element count, parents
// pointing at earlier document/array elements).
#include <cstdio>
#include <cstdint>
#include <random>
#include <vector>

#include "fedavg_hip.h"

static int64_t walk(const uint8_t* b, int64_t n, int64_t off, int depth) {
    if (depth > 100) return -1;
    uint8_t ty[256], st[256];
    int64_t no[256], vo[256], vl[256];
    int32_t nl[256];
    int64_t k = fa_bson_elements(b, n, off, ty, no, nl, vo, vl, st, 256);
    if (k < 0) return k;
    int64_t total = k;
    for (int64_t i = 0; i < k && i < 256; ++i) {
        if (no[i] < 0 || no[i] + nl[i] > n || vo[i] < 0 || vl[i] < 0 || vo[i] + vl[i] > n) {
            std::fprintf(stderr, "out-of-range element %lld\n", (long long)i);
            std::abort();
        }
        if (ty[i] == 0x03 || ty[i] == 0x04) {
            int64_t r = walk(b, n, vo[i], depth + 1);
            if (r < 0) return r;
            total += r;
        }
    }
    return total;
}

static int64_t both(const uint8_t* b, int64_t n) {
    const int64_t r = walk(b, n, 0, 0);
    static uint8_t ty[4096], st[4096];
    static int32_t pa[4096], nl[4096];
    static int64_t no[4096], vo[4096], vl[4096];
    const int64_t w = fa_bson_walk(b, n, 0, ty, pa, no, nl, vo, vl, st, 4096);
    if ((r < 0) != (w < 0) || (r >= 0 && r != w)) {
        std::fprintf(stderr, "walk mismatch: levels %lld, tree %lld\n", (long long)r, (long long)w);
        std::abort();
    }
    for (int64_t k = 0; k < w && k < 4096; ++k)
        if (pa[k] >= k || (pa[k] >= 0 && ty[pa[k]] != 0x03 && ty[pa[k]] != 0x04) || vo[k] + vl[k] > n) {
            std::fprintf(stderr, "bad tree element %lld\n", (long long)k);
            std::abort();
        }
    return r;
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<uint8_t> seed(1 << 20);
    size_t n = std::fread(seed.data(), 1, seed.size(), f);
    std::fclose(f);
    seed.resize(n);
    long ok = 0, bad = 0;
    for (size_t cut = 0; cut <= n; ++cut) {
        std::vector<uint8_t> c(seed.begin(), seed.begin() + cut);  // exact-size heap buffer
        (both(c.data(), (int64_t)cut) >= 0 ? ok : bad)++;
    }
    std::mt19937 rng(7);
    for (int it = 0; it < 300000; ++it) {
        std::vector<uint8_t> c = seed;
        for (int j = 0, m = 1 + rng() % 4; j < m; ++j) c[rng() % n] = (uint8_t)rng();
        (both(c.data(), (int64_t)n) >= 0 ? ok : bad)++;
    }
    std::printf("bson fuzz: %ld accepted, %ld rejected, seed walk = %lld elements\n", ok, bad,
                (long long)both(seed.data(), (int64_t)n));
    return 0;
}
