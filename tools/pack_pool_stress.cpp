#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>
#include <thread>
#include <random>
extern "C" int fa_pack(void*, const int64_t*, const void* const*, const int64_t*, int64_t, int);
int main() {
  std::mt19937 rng(3);
  auto worker = [](int seed) {
    std::mt19937 r(seed);
    for (int it = 0; it < 300; ++it) {
      int n = 1 + r() % 7;
      std::vector<std::vector<uint8_t>> src(n);
      std::vector<const void*> ptr(n); std::vector<int64_t> sz(n), off(n);
      int64_t pos = 0;
      for (int i = 0; i < n; ++i) { src[i].resize((r() % 3) ? r() % (6 << 20) : r() % 100); for (auto& b : src[i]) b = r(); ptr[i] = src[i].data(); sz[i] = src[i].size(); pos += r() % 64; off[i] = pos; pos += sz[i]; }
      std::vector<uint8_t> dst(pos + 1, 0);
      if (fa_pack(dst.data(), off.data(), ptr.data(), sz.data(), n, 1 + r() % 16)) { printf("err\n"); exit(1); }
      for (int i = 0; i < n; ++i) if (sz[i] && memcmp(dst.data() + off[i], src[i].data(), sz[i])) { printf("mismatch\n"); exit(1); }
    }
  };
  std::thread a(worker, 1), b(worker, 2); a.join(); b.join();
  printf("pack ok\n");
}
