// hbm_probe — measure achievable HBM read bandwidth on MI355X for several
// access patterns, to calibrate the fold's roofline (not part of the product).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/build/hbm_probe tools/hbm_probe.hip
//   tools/build/hbm_probe [GiB]
//
// Patterns (all read every byte of the buffer exactly once per launch):
//   sweep   grid-stride over the whole buffer, 8 x 16 B loads in flight per lane
//   chunk   each block streams its own contiguous chunk, 8 x 16 B per lane per step
//   fold2d  the fold's shape: rows x cols fp32, a block reads C*4 KiB of every row
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e = (x);                                                                    \
        if (e != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));           \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

template <bool NT>
__device__ __forceinline__ f32x4 ld(const f32x4* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}

template <bool NT, int K>
__global__ __launch_bounds__(256) void sweep(const f32x4* __restrict__ X, int64_t nq, float* sink) {
    f32x4 acc = {0, 0, 0, 0};
    const int64_t stride = (int64_t)gridDim.x * 256;
    int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; q + (K - 1) * stride < nq; q += K * stride) {
        f32x4 v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = ld<NT>(X + q + k * stride);
#pragma unroll
        for (int k = 0; k < K; ++k) acc += v[k];
    }
    for (; q < nq; q += stride) acc += ld<NT>(X + q);
    if (acc.x + acc.y + acc.z + acc.w == 123.456f) sink[0] = acc.x;  // keep loads live
}

template <bool NT>
__global__ __launch_bounds__(256) void chunk(const f32x4* __restrict__ X, int64_t nq, int64_t per, float* sink) {
    f32x4 acc = {0, 0, 0, 0};
    const int64_t lo = (int64_t)blockIdx.x * per, hi = lo + per < nq ? lo + per : nq;
    int64_t q = lo + threadIdx.x;
    for (; q + 7 * 256 < hi; q += 8 * 256) {
        f32x4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = ld<NT>(X + q + k * 256);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += v[k];
    }
    for (; q < hi; q += 256) acc += ld<NT>(X + q);
    if (acc.x + acc.y + acc.z + acc.w == 123.456f) sink[0] = acc.x;
}

template <int U, int C>
__global__ __launch_bounds__(256) void fold2d(const f32x4* __restrict__ X, int64_t rows, int64_t ldq, float* sink) {
    const int64_t q0 = (int64_t)blockIdx.x * (256 * C) + threadIdx.x;
    f32x4 acc[C];
#pragma unroll
    for (int c = 0; c < C; ++c) acc[c] = f32x4{0, 0, 0, 0};
    for (int64_t i = 0; i + U <= rows; i += U) {
        f32x4 v[U][C];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int c = 0; c < C; ++c) v[u][c] = __builtin_nontemporal_load(X + (i + u) * ldq + q0 + c * 256);
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int c = 0; c < C; ++c) acc[c] += v[u][c];
    }
    float t = 0;
#pragma unroll
    for (int c = 0; c < C; ++c) t += acc[c].x + acc[c].y + acc[c].z + acc[c].w;
    if (t == 123.456f) sink[0] = t;
}

// fold2d plus the real fold's extra work, to bisect the gap to the product
// kernel: W = multiply by a per-row weight read through the scalar cache,
// S = store the [cols] result.
template <int U, int C, bool W, int S>
__global__ __launch_bounds__(256) void fold2d_x(const f32x4* __restrict__ X, int64_t rows, int64_t ldq,
                                                 const float* __restrict__ w, f32x4* __restrict__ out,
                                                 float* sink) {
    const int64_t q0 = (int64_t)blockIdx.x * (256 * C) + threadIdx.x;
    f32x4 acc[C];
#pragma unroll
    for (int c = 0; c < C; ++c) acc[c] = f32x4{0, 0, 0, 0};
    for (int64_t i = 0; i + U <= rows; i += U) {
        f32x4 v[U][C];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int c = 0; c < C; ++c) v[u][c] = __builtin_nontemporal_load(X + (i + u) * ldq + q0 + c * 256);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float wi = W ? w[i + u] : 1.0f;
#pragma unroll
            for (int c = 0; c < C; ++c) acc[c] += W ? v[u][c] * wi : v[u][c];
        }
    }
    if constexpr (S == 1) {
#pragma unroll
        for (int c = 0; c < C; ++c) out[q0 + c * 256] = acc[c];
    } else if constexpr (S == 2) {
#pragma unroll
        for (int c = 0; c < C; ++c) __builtin_nontemporal_store(acc[c], out + q0 + c * 256);
    } else {
        float t = 0;
#pragma unroll
        for (int c = 0; c < C; ++c) t += acc[c].x + acc[c].y + acc[c].z + acc[c].w;
        if (t == 123.456f) sink[0] = t;
    }
}

// tiled layout [P/T][rows][T]: block b owns tile b; rows of a tile are adjacent,
// so a block streams rows*T*4 contiguous bytes.  T = 256*C*4 floats.
template <int U, int C>
__global__ __launch_bounds__(256) void fold_tiled(const f32x4* __restrict__ X, int64_t rows, float* sink) {
    constexpr int TQ = 256 * C;  // quads per tile row
    const f32x4* base = X + (int64_t)blockIdx.x * rows * TQ + threadIdx.x;
    f32x4 acc[C];
#pragma unroll
    for (int c = 0; c < C; ++c) acc[c] = f32x4{0, 0, 0, 0};
    for (int64_t i = 0; i + U <= rows; i += U) {
        f32x4 v[U][C];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int c = 0; c < C; ++c) v[u][c] = __builtin_nontemporal_load(base + (i + u) * TQ + c * 256);
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int c = 0; c < C; ++c) acc[c] += v[u][c];
    }
    float t = 0;
#pragma unroll
    for (int c = 0; c < C; ++c) t += acc[c].x + acc[c].y + acc[c].z + acc[c].w;
    if (t == 123.456f) sink[0] = t;
}

// tiled layout with the fold's extras (per-row weights, non-temporal output store)
template <int U, int C>
__global__ __launch_bounds__(256) void fold_tiled_x(const f32x4* __restrict__ X, int64_t rows,
                                                     const float* __restrict__ w, f32x4* __restrict__ out) {
    constexpr int TQ = 256 * C;
    const f32x4* base = X + (int64_t)blockIdx.x * rows * TQ + threadIdx.x;
    f32x4 acc[C];
#pragma unroll
    for (int c = 0; c < C; ++c) acc[c] = f32x4{0, 0, 0, 0};
    for (int64_t i = 0; i + U <= rows; i += U) {
        f32x4 v[U][C];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int c = 0; c < C; ++c) v[u][c] = __builtin_nontemporal_load(base + (i + u) * TQ + c * 256);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float wi = w[i + u];
#pragma unroll
            for (int c = 0; c < C; ++c) acc[c] += v[u][c] * wi;
        }
    }
#pragma unroll
    for (int c = 0; c < C; ++c)
        __builtin_nontemporal_store(acc[c], out + (int64_t)blockIdx.x * TQ + threadIdx.x + c * 256);
}

__global__ void fill(f32x4* X, int64_t nq) {
    for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < nq; q += (int64_t)gridDim.x * 256)
        X[q] = f32x4{1.f, 2.f, 3.f, (float)(q & 1023)};
}

template <typename F>
double time_ms(F launch, int reps = 7) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    launch();
    launch();
    CK(hipDeviceSynchronize());
    float best[16];
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(a));
        launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&best[r], a, b));
    }
    // median
    for (int i = 0; i < reps; ++i)
        for (int j = i + 1; j < reps; ++j)
            if (best[j] < best[i]) { float t = best[i]; best[i] = best[j]; best[j] = t; }
    return best[reps / 2];
}

int main(int argc, char** argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 38.0;
    const int64_t rows = argc > 2 ? atoll(argv[2]) : 1024;
    const bool pitch_only = argc > 3 && argv[3][0] == 'p';
    const int64_t cols = (int64_t)(gib * (1ll << 30) / 4 / rows) / 4096 * 4096;
    const int64_t nq = rows * cols / 4;
    const double bytes = (double)nq * 16;
    f32x4* X;
    float* sink;
    CK(hipMalloc(&X, (size_t)bytes));
    CK(hipMalloc(&sink, 64));
    hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, X, nq);
    CK(hipDeviceSynchronize());
    printf("buffer %.2f GB (%lld rows x %lld cols fp32)\n", bytes / 1e9, (long long)rows, (long long)cols);
    auto report = [&](const char* name, double ms) {
        printf("%-28s %8.3f ms  %8.1f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    if (pitch_only) {
        // same fold-shaped read, row pitch padded by `pad` quads (buffer has slack)
        const int64_t ldq0 = cols / 4;
        const int64_t slack = 65536 + 64;         // quads per row kept free for padding
        const int64_t ncol_q = (ldq0 - slack) / 1024 * 1024;  // quads actually read per row
        for (int64_t pad : {0, 16, 64, 256, 1024, 4096, 16384, 65536}) {
            const int64_t ldq = ncol_q + pad;
            // host-side bounds check before any launch: the last row must end inside the buffer
            if ((rows - 1) * ldq + ncol_q > nq) {
                fprintf(stderr, "pad %lld would overrun the buffer; skipped\n", (long long)pad);
                continue;
            }
            char nm[64];
            snprintf(nm, sizeof nm, "fold2d u8c4 pitch+%lldB", (long long)(pad * 16));
            const double rb = (double)rows * ncol_q * 16;
            double ms = time_ms([&] {
                hipLaunchKernelGGL((fold2d<8, 4>), dim3(ncol_q / 1024), dim3(256), 0, 0, X, rows, ldq, sink); });
            printf("%-28s %8.3f ms  %8.1f GB/s\n", nm, ms, rb / (ms * 1e-3) / 1e9);
            fflush(stdout);
        }
        CK(hipFree(X));
        return 0;
    }
    for (int g : {1024, 2048, 4096, 8192, 16384, 65535}) {
        char nm[64];
        snprintf(nm, sizeof nm, "sweep nt k8 grid %d", g);
        report(nm, time_ms([&] { hipLaunchKernelGGL((sweep<true, 8>), dim3(g), dim3(256), 0, 0, X, nq, sink); }));
    }
    report("sweep plain k8 grid 8192",
           time_ms([&] { hipLaunchKernelGGL((sweep<false, 8>), dim3(8192), dim3(256), 0, 0, X, nq, sink); }));
    report("sweep nt k16 grid 4096",
           time_ms([&] { hipLaunchKernelGGL((sweep<true, 16>), dim3(4096), dim3(256), 0, 0, X, nq, sink); }));
    report("sweep nt k4 grid 16384",
           time_ms([&] { hipLaunchKernelGGL((sweep<true, 4>), dim3(16384), dim3(256), 0, 0, X, nq, sink); }));
    for (int64_t kb : {16, 64, 256, 1024, 4096}) {
        int64_t per = kb * 1024 / 16;
        int64_t grid = (nq + per - 1) / per;
        char nm[64];
        snprintf(nm, sizeof nm, "chunk nt %lld KiB/block", (long long)kb);
        report(nm, time_ms([&] { hipLaunchKernelGGL((chunk<true>), dim3(grid), dim3(256), 0, 0, X, nq, per, sink); }));
    }
    const int64_t ldq = cols / 4;
    {
        float* w;
        f32x4* o;
        CK(hipMalloc(&w, rows * sizeof(float)));
        CK(hipMalloc(&o, ldq * sizeof(f32x4)));
        std::vector<float> hw(rows, 3.0f);
        CK(hipMemcpy(w, hw.data(), rows * sizeof(float), hipMemcpyHostToDevice));
        report("fold2d_x u8c4 (read only)", time_ms([&] {
            hipLaunchKernelGGL((fold2d_x<8, 4, false, 0>), dim3(ldq / 1024), dim3(256), 0, 0, X, rows, ldq, w, o, sink); }));
        report("fold2d_x u8c4 +weights", time_ms([&] {
            hipLaunchKernelGGL((fold2d_x<8, 4, true, 0>), dim3(ldq / 1024), dim3(256), 0, 0, X, rows, ldq, w, o, sink); }));
        report("fold2d_x u8c4 +store", time_ms([&] {
            hipLaunchKernelGGL((fold2d_x<8, 4, false, 1>), dim3(ldq / 1024), dim3(256), 0, 0, X, rows, ldq, w, o, sink); }));
        report("fold2d_x u8c4 +weights+store", time_ms([&] {
            hipLaunchKernelGGL((fold2d_x<8, 4, true, 1>), dim3(ldq / 1024), dim3(256), 0, 0, X, rows, ldq, w, o, sink); }));
        report("fold2d_x u8c4 +weights+ntstore", time_ms([&] {
            hipLaunchKernelGGL((fold2d_x<8, 4, true, 2>), dim3(ldq / 1024), dim3(256), 0, 0, X, rows, ldq, w, o, sink); }));
        report("fold2d_x u4c1 +weights+store", time_ms([&] {
            hipLaunchKernelGGL((fold2d_x<4, 1, true, 1>), dim3(ldq / 256), dim3(256), 0, 0, X, rows, ldq, w, o, sink); }));
        report("fold2d_x u4c1 read only", time_ms([&] {
            hipLaunchKernelGGL((fold2d_x<4, 1, false, 0>), dim3(ldq / 256), dim3(256), 0, 0, X, rows, ldq, w, o, sink); }));
        report("tiled_x u8c1 +w+nts (T=4KiB)", time_ms([&] {
            hipLaunchKernelGGL((fold_tiled_x<8, 1>), dim3(ldq / 256), dim3(256), 0, 0, X, rows, w, o); }));
        report("tiled_x u4c2 +w+nts (T=8KiB)", time_ms([&] {
            hipLaunchKernelGGL((fold_tiled_x<4, 2>), dim3(ldq / 512), dim3(256), 0, 0, X, rows, w, o); }));
        report("tiled_x u8c4 +w+nts (T=16KiB)", time_ms([&] {
            hipLaunchKernelGGL((fold_tiled_x<8, 4>), dim3(ldq / 1024), dim3(256), 0, 0, X, rows, w, o); }));
        report("fold2d_x u8c4 +w+nts (again)", time_ms([&] {
            hipLaunchKernelGGL((fold2d_x<8, 4, true, 2>), dim3(ldq / 1024), dim3(256), 0, 0, X, rows, ldq, w, o, sink); }));
        CK(hipFree(w));
        CK(hipFree(o));
    }
    report("fold2d u4c4", time_ms([&] {
        hipLaunchKernelGGL((fold2d<4, 4>), dim3(ldq / 1024), dim3(256), 0, 0, X, rows, ldq, sink); }));
    report("fold2d u4c2", time_ms([&] {
        hipLaunchKernelGGL((fold2d<4, 2>), dim3(ldq / 512), dim3(256), 0, 0, X, rows, ldq, sink); }));
    report("fold2d u4c1", time_ms([&] {
        hipLaunchKernelGGL((fold2d<4, 1>), dim3(ldq / 256), dim3(256), 0, 0, X, rows, ldq, sink); }));
    report("fold2d u8c4", time_ms([&] {
        hipLaunchKernelGGL((fold2d<8, 4>), dim3(ldq / 1024), dim3(256), 0, 0, X, rows, ldq, sink); }));
    report("fold2d u8c2", time_ms([&] {
        hipLaunchKernelGGL((fold2d<8, 2>), dim3(ldq / 512), dim3(256), 0, 0, X, rows, ldq, sink); }));
    report("fold2d u16c1", time_ms([&] {
        hipLaunchKernelGGL((fold2d<16, 1>), dim3(ldq / 256), dim3(256), 0, 0, X, rows, ldq, sink); }));
    report("tiled u4c1 (T=4KiB)", time_ms([&] {
        hipLaunchKernelGGL((fold_tiled<4, 1>), dim3(ldq / 256), dim3(256), 0, 0, X, rows, sink); }));
    report("tiled u8c1 (T=4KiB)", time_ms([&] {
        hipLaunchKernelGGL((fold_tiled<8, 1>), dim3(ldq / 256), dim3(256), 0, 0, X, rows, sink); }));
    report("tiled u4c2 (T=8KiB)", time_ms([&] {
        hipLaunchKernelGGL((fold_tiled<4, 2>), dim3(ldq / 512), dim3(256), 0, 0, X, rows, sink); }));
    report("tiled u4c4 (T=16KiB)", time_ms([&] {
        hipLaunchKernelGGL((fold_tiled<4, 4>), dim3(ldq / 1024), dim3(256), 0, 0, X, rows, sink); }));
    report("tiled u2c4 (T=16KiB)", time_ms([&] {
        hipLaunchKernelGGL((fold_tiled<2, 4>), dim3(ldq / 1024), dim3(256), 0, 0, X, rows, sink); }));
    report("tiled u8c4 (T=16KiB)", time_ms([&] {
        hipLaunchKernelGGL((fold_tiled<8, 4>), dim3(ldq / 1024), dim3(256), 0, 0, X, rows, sink); }));
    CK(hipFree(X));
    return 0;
}
