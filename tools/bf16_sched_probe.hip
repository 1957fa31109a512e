// bf16_sched_probe.hip -- load-schedule probe for the bf16 fold's tile body
// (fold_octets in csrc/fold_kernels.hpp), standalone so a schedule costs one
// 20-second compile instead of a library build.  Every variant folds the same
// [N x P] bf16 rows with the same per-column in-order left fold (separate
// multiply and add, fp-contract off) as the library, so every output bit must
// equal the first variant's; the probe checks that and prints one line per
// variant: median ms over the launches, GB/s of algorithmic bytes.
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 tools/bf16_sched_probe.hip -o /tmp/bsp
//   /tmp/bsp [N] [P] [reps]
// Schedules (one lane owns C octets spaced 256 lanes apart, as the library):
//   grp   U rows x C octets loaded as a group, then added (the library's form)
//   grpb  the same with a scheduling barrier after the group's loads
//   roll  software pipeline across groups: a ring of R rows in flight, row i's
//         slot reloaded with row i + R right after row i is added
//   dbl   two groups of U rows: group g+1's loads issued before group g's adds
//   chunk G rows straight-line (no loop-carried loads, which the compiler
//         drains with vmcnt(0) at the back-edge), inside them a ring of U rows
//         in flight: row u + U issued as row u is added, a scheduling barrier
//         per row keeps the order; one drain per G rows
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#pragma clang fp contract(off)

#define CHECK(x)                                                                            \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                        \
        }                                                                                   \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kB = 256;

__device__ __forceinline__ void unpack(u32x4 w, f32x4& e, f32x4& o) {
    e = __builtin_bit_cast(f32x4, w << 16);
    o = __builtin_bit_cast(f32x4, w & 0xFFFF0000u);
}
__device__ __forceinline__ u32x4 ld(const u32x4* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ uint32_t f2bf(float f) {
    uint32_t u = __float_as_uint(f);
    if (f != f) return (u >> 16) | 0x40u;
    return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}

template <int C>
__device__ __forceinline__ void add_row(f32x4 (&ev)[C], f32x4 (&od)[C], const u32x4 (&v)[C], float ai) {
#pragma unroll
    for (int c = 0; c < C; ++c) {
        f32x4 e, o;
        unpack(v[c], e, o);
        ev[c] = ev[c] + e * ai;
        od[c] = od[c] + o * ai;
    }
}

enum { GRP = 0, GRPB = 1, ROLL = 2, DBL = 3, CHUNK = 4, OUTB = 16 };  // OUTB: also the RNE bf16 copy

template <int U, int C, int MODE, int G = 0>
__device__ __forceinline__ void fold(const u32x4* __restrict__ p, int64_t ldo, int64_t N, const float* __restrict__ a,
                                     float div, float* __restrict__ out, int64_t o0, uint16_t* __restrict__ outb) {
    constexpr int M = MODE & 15;
    f32x4 ev[C], od[C];
    {
        const float a0 = a[0];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            f32x4 e, o;
            unpack(ld(p + c * kB), e, o);
            ev[c] = e * a0;
            od[c] = o * a0;
        }
    }
    int64_t i = 1;
    if constexpr (M == GRP || M == GRPB) {
        for (; i + U <= N; i += U) {
            u32x4 v[U][C];
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int c = 0; c < C; ++c) v[u][c] = ld(p + (i + u) * ldo + c * kB);
            if constexpr (M == GRPB) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < U; ++u) add_row<C>(ev, od, v[u], a[i + u]);
        }
    } else if constexpr (M == ROLL) {
        // ring of U rows: rows i .. i+U-1 in flight on entry of each group
        if (N - 1 >= 2 * U) {
            u32x4 v[U][C];
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int c = 0; c < C; ++c) v[u][c] = ld(p + (i + u) * ldo + c * kB);
            for (; i + 2 * U <= N; i += U) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    u32x4 x[C];
#pragma unroll
                    for (int c = 0; c < C; ++c) x[c] = v[u][c];
#pragma unroll
                    for (int c = 0; c < C; ++c) v[u][c] = ld(p + (i + u + U) * ldo + c * kB);
                    add_row<C>(ev, od, x, a[i + u]);
                }
            }
            // the last loaded group
#pragma unroll
            for (int u = 0; u < U; ++u) add_row<C>(ev, od, v[u], a[i + u]);
            i += U;
        }
    } else if constexpr (M == CHUNK) {
        static_assert(G % U == 0 && G >= 2 * U, "chunk of whole rings");
        for (; i + G <= N; i += G) {
            u32x4 v[U][C];
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int c = 0; c < C; ++c) v[u][c] = ld(p + (i + u) * ldo + c * kB);
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const int u = g % U;
                u32x4 x[C];
#pragma unroll
                for (int c = 0; c < C; ++c) x[c] = v[u][c];
                if (g + U < G) {
#pragma unroll
                    for (int c = 0; c < C; ++c) v[u][c] = ld(p + (i + g + U) * ldo + c * kB);
                }
                add_row<C>(ev, od, x, a[i + g]);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        for (; i + 4 <= N; i += 4) {  // the rows past the last chunk, 4 at a time
            u32x4 v[4][C];
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int c = 0; c < C; ++c) v[u][c] = ld(p + (i + u) * ldo + c * kB);
#pragma unroll
            for (int u = 0; u < 4; ++u) add_row<C>(ev, od, v[u], a[i + u]);
        }
    } else {  // DBL: group g+1 loaded before group g's adds
        if (N - 1 >= 2 * U) {
            u32x4 v0[U][C], v1[U][C];
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int c = 0; c < C; ++c) v0[u][c] = ld(p + (i + u) * ldo + c * kB);
            for (; i + 3 * U <= N; i += 2 * U) {
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int c = 0; c < C; ++c) v1[u][c] = ld(p + (i + U + u) * ldo + c * kB);
#pragma unroll
                for (int u = 0; u < U; ++u) add_row<C>(ev, od, v0[u], a[i + u]);
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int c = 0; c < C; ++c) v0[u][c] = ld(p + (i + 2 * U + u) * ldo + c * kB);
#pragma unroll
                for (int u = 0; u < U; ++u) add_row<C>(ev, od, v1[u], a[i + U + u]);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) add_row<C>(ev, od, v0[u], a[i + u]);
            i += U;
        }
    }
    for (; i < N; ++i) {
        u32x4 v[C];
#pragma unroll
        for (int c = 0; c < C; ++c) v[c] = ld(p + i * ldo + c * kB);
        add_row<C>(ev, od, v, a[i]);
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const f32x4 e = ev[c] / div, o = od[c] / div;
        f32x4* o4 = reinterpret_cast<f32x4*>(out) + 2 * (o0 + (int64_t)c * kB);
        __builtin_nontemporal_store(f32x4{e.x, o.x, e.y, o.y}, o4);
        __builtin_nontemporal_store(f32x4{e.z, o.z, e.w, o.w}, o4 + 1);
        if constexpr ((MODE & OUTB) != 0) {
            u32x4 b;
            b.x = f2bf(e.x) | (f2bf(o.x) << 16);
            b.y = f2bf(e.y) | (f2bf(o.y) << 16);
            b.z = f2bf(e.z) | (f2bf(o.z) << 16);
            b.w = f2bf(e.w) | (f2bf(o.w) << 16);
            __builtin_nontemporal_store(b, reinterpret_cast<u32x4*>(outb) + o0 + (int64_t)c * kB);
        }
    }
}

// grid-stride over tiles of kB lanes x C octets; P a multiple of 8 * kB * C
template <int U, int C, int MODE, int WPE, int G = 0>
__global__ __launch_bounds__(kB, WPE) void k_probe(const uint16_t* __restrict__ X, int64_t N, int64_t ldx,
                                                   const float* __restrict__ a, float div, float* __restrict__ out,
                                                   int64_t ntiles, uint16_t* __restrict__ outb) {
    const u32x4* X8 = reinterpret_cast<const u32x4*>(X);
    const int64_t ldo = ldx >> 3;
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int64_t o0 = t * (kB * C) + threadIdx.x;
        fold<U, C, MODE, G>(X8 + o0, ldo, N, a, div, out, o0, outb);
    }
}

__global__ void k_synth(uint16_t* X, int64_t n, uint64_t seed) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        // finite bf16 in about [-2, 2]: sign, exponent 0x70..0x7F, mantissa bits
        X[i] = (uint16_t)(((z >> 8) & 0x8000u) | ((0x70u + ((z >> 20) & 0xFu)) << 7) | (z & 0x7Fu));
    }
}

struct Variant {
    const char* name;
    int C;
    int per_cu;  // blocks per CU in the grid
    void (*launch)(dim3, hipStream_t, const uint16_t*, int64_t, int64_t, const float*, float, float*, int64_t,
                   uint16_t*);
    int bands = 1;  // launches over contiguous column bands (the library's band forms)
};

template <int U, int C, int MODE, int WPE, int G = 0>
void launch_v(dim3 g, hipStream_t st, const uint16_t* X, int64_t N, int64_t ldx, const float* a, float div, float* out,
              int64_t nt, uint16_t* outb) {
    hipLaunchKernelGGL((k_probe<U, C, MODE, WPE, G>), g, dim3(kB), 0, st, X, N, ldx, a, div, out, nt, outb);
}

#define V(name, U, C, MODE, PER, NB) {name, C, PER, launch_v<U, C, MODE, PER>, NB}
#define VC(name, U, C, G, PER, NB) {name, C, PER, launch_v<U, C, CHUNK | OUTB, PER, G>, NB}
// _ob: the RNE bf16 copy stored too (as the library); _bN: N launches over
// contiguous column bands (the library's band forms: bands of <= 4 passes)
static const Variant kVariants[] = {
    V("grp_u8c4", 8, 4, GRP, 1, 1),
    V("grp_u8c4_ob", 8, 4, GRP | OUTB, 1, 1),
    V("grp_u8c4_ob_b2", 8, 4, GRP | OUTB, 1, 2),
    V("grp_u8c2_ob_b3", 8, 2, GRP | OUTB, 1, 3),
    V("grp_u8c2_ob", 8, 2, GRP | OUTB, 1, 1),
    V("roll_u8c4_ob", 8, 4, ROLL | OUTB, 1, 1),
    V("roll_u8c4_ob_b2", 8, 4, ROLL | OUTB, 1, 2),
    VC("chunk64_r4c4_ob", 4, 4, 64, 1, 1),
    VC("chunk64_r4c4_ob_b2", 4, 4, 64, 1, 2),
    V("grp_u4c4_x2_ob", 4, 4, GRP | OUTB, 2, 1),
    V("grp_u8c4_ob_b3", 8, 4, GRP | OUTB, 1, 3),
    V("grp_u8c4", 8, 4, GRP, 1, 1),
    V("grp_u8c4_ob_b2", 8, 4, GRP | OUTB, 1, 2),
    V("grp_u8c2_ob_b3", 8, 2, GRP | OUTB, 1, 3),
};

int main(int argc, char** argv) {
    const int64_t N = argc > 1 ? atoll(argv[1]) : 256;
    const int64_t P0 = argc > 2 ? atoll(argv[2]) : 4934912;
    const int reps = argc > 3 ? atoi(argv[3]) : 20;
    const int64_t unit = 8 * kB * 4;  // every variant's tiles divide P
    const int64_t P = (P0 / unit) * unit, ldx = P;
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    uint16_t* X;
    float *a, *out, *ref;
    uint16_t* outb;
    CHECK(hipMalloc(&X, (size_t)N * ldx * 2));
    CHECK(hipMalloc(&a, N * 4));
    CHECK(hipMalloc(&out, P * 4));
    CHECK(hipMalloc(&ref, P * 4));
    CHECK(hipMalloc(&outb, P * 2));
    hipLaunchKernelGGL(k_synth, dim3(4096), dim3(256), 0, 0, X, N * ldx, 12345ull);
    std::vector<float> ha(N);
    double tot = 0;
    for (int64_t i = 0; i < N; ++i) tot += (ha[i] = (float)(1 + (i * 7919) % 97));
    CHECK(hipMemcpy(a, ha.data(), N * 4, hipMemcpyHostToDevice));
    const float div = (float)tot;
    hipStream_t st;
    CHECK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const double bytes = (double)N * P * 2 + (double)P * 6;  // the f32 result and its bf16 copy
    printf("N %lld P %lld (%.3f GB per launch), %d CUs, %d reps\n", (long long)N, (long long)P, bytes / 1e9, cus, reps);
    std::vector<uint32_t> h0(P), h1(P);
    bool have_ref = false;
    for (const Variant& v : kVariants) {
        const int64_t to = (int64_t)kB * v.C;                  // octets per tile
        const int64_t tiles = P / 8 / to;
        const int64_t band_tiles = (tiles + v.bands - 1) / v.bands;
        auto launch = [&]() {
            for (int64_t t0 = 0; t0 < tiles; t0 += band_tiles) {
                const int64_t nt = std::min(band_tiles, tiles - t0);
                const int64_t slots = (int64_t)cus * v.per_cu;
                const int64_t passes = (nt + slots - 1) / slots;
                const int64_t grid = (nt + passes - 1) / passes;  // balanced passes
                const int64_t c0 = t0 * to * 8;                    // first column of the band
                v.launch(dim3((unsigned)grid), st, X + c0, N, ldx, a, div, out + c0, nt, outb + c0);
            }
        };
        CHECK(hipMemsetAsync(out, 0xFF, P * 4, st));
        launch();  // untimed
        CHECK(hipGetLastError());
        CHECK(hipStreamSynchronize(st));
        CHECK(hipMemcpy(have_ref ? h1.data() : h0.data(), out, P * 4, hipMemcpyDeviceToHost));
        bool same = true;
        if (have_ref) same = memcmp(h0.data(), h1.data(), P * 4) == 0;
        have_ref = true;
        std::vector<float> ms;
        for (int r = 0; r < reps; ++r) {
            CHECK(hipEventRecord(e0, st));
            launch();
            CHECK(hipEventRecord(e1, st));
            CHECK(hipEventSynchronize(e1));
            float t;
            CHECK(hipEventElapsedTime(&t, e0, e1));
            ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        const float med = ms[ms.size() / 2];
        printf("%-20s %d band(s): median %.4f ms (min %.4f)  %.1f GB/s  bits %s\n", v.name, v.bands, med, ms[0],
               bytes / med / 1e6, same ? "same" : "DIFFER");
        fflush(stdout);
    }
    return 0;
}
