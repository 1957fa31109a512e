#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <random>
extern "C" int fa_npz_index(const uint8_t*, int64_t, int64_t*, int64_t*, int32_t*, int32_t*, int64_t*, int);
int main() {
  FILE* f = fopen("a.npz", "rb"); std::vector<uint8_t> b(1 << 20); size_t n = fread(b.data(), 1, b.size(), f); b.resize(n);
  int64_t off[64], cnt[64], shp[64*8]; int32_t dt[64], nd[64];
  int ok = 0;
  for (size_t cut = 0; cut <= n; ++cut) { std::vector<uint8_t> c(b.begin(), b.begin() + cut); ok += fa_npz_index(c.data(), cut, off, cnt, dt, nd, shp, 64) >= 0; }
  std::mt19937 rng(1);
  for (int it = 0; it < 200000; ++it) { std::vector<uint8_t> c = b; int k = 1 + rng() % 4; for (int j = 0; j < k; ++j) c[rng() % n] = rng(); ok += fa_npz_index(c.data(), n, off, cnt, dt, nd, shp, 64) >= 0; }
  printf("ok parses %d, full=%d\n", ok, fa_npz_index(b.data(), n, off, cnt, dt, nd, shp, 64));
}
